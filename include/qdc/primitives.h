/*
 * qdc/primitives.h — the drop-in C ABI of the state-vector hot path.
 *
 * These are exactly the 18 `extern "C"` entry points that the reference's Rust
 * layer binds in src/primitives_bind.rs:15-119 (implemented for CUDA in
 * src/primitives.cu:141-953).  Here they are implemented by hand-written HIP
 * kernels for gfx950 (libqdc_f32.so / libqdc_f64.so).  One precision per
 * library, exactly like the reference's Cargo feature `f64` (Cargo.toml:25-27,
 * build.rs:17-20): compile against this header with -DQDC_F64 to get the
 * double-precision layout.
 *
 * Conventions shared with the reference (SURVEY.md §8 a/b):
 *   - a state is a device buffer of 2^n interleaved {re, im} amplitudes;
 *     amplitude index bit k = qubit k (qubit 0 least significant);
 *   - gate / density / gradient pointers are HOST memory, read or written
 *     before the call returns;
 *   - densities and gradients are ACCUMULATED (`+=`) into the caller's buffer
 *     (src/primitives.cu:281-288, 384-391, 482-489, 765-772, 865-872);
 *   - NULL return = success, otherwise a NUL-terminated message owned by the
 *     library (thread-local storage: valid until the next failing call on the
 *     same thread; never free it).
 *
 * Differences that only remove reference defects: every size is computed in
 * 64-bit (the reference's `1 << qubits_number` is `int`, so it is limited to
 * n <= 30, src/primitives.cu:147); gates are kernel arguments, not global
 * `__constant__` symbols, so concurrent callers do not race (README.md:13);
 * every launch is error-checked.
 */
#ifndef QDC_PRIMITIVES_H
#define QDC_PRIMITIVES_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#ifdef QDC_F64
typedef double qdc_real;
#else
typedef float qdc_real;
#endif

/* Layout-equal to num_complex::Complex<f32|f64> (#[repr(C)]), used by the
 * reference as `Complex` (src/primitives_bind.rs:10-13). */
typedef struct qdc_complex {
  qdc_real re;
  qdc_real im;
} qdc_complex;

/* |0...0>.  replaces src/primitives.cu:189-199 (binding pb.rs:16-19). */
void set2standard(qdc_complex* state, size_t qubits_number);

/* Allocate an uninitialised 2^n state.  replaces pr.cu:141-150 (pb.rs:20-23). */
const char* get_state(qdc_complex** state, size_t qubits_number);

/* Free a state.  replaces pr.cu:166-173 (pb.rs:24). */
const char* drop_state(qdc_complex* state);

/* Device -> host copy of 2^n amplitudes.  replaces pr.cu:153-163 (pb.rs:25-29). */
const char* copy_to_host(const qdc_complex* state, qdc_complex* host_state,
                         size_t qubits_number);

/* Host -> device copy of 2^n amplitudes.  replaces pr.cu:496-510 (pb.rs:63-67). */
const char* set_from_host(qdc_complex* device_state, const qdc_complex* host_state,
                          size_t qubits_number);

/* psi <- (U on qubit pos) psi, U row-major 2x2: out[p] = sum_q U[2p+q] in[q].
 * replaces pr.cu:513-545 (pb.rs:30-35). */
const char* q1gate(qdc_complex* state, const qdc_complex* gate, size_t pos,
                   size_t qubits_number);

/* psi <- U^-1 psi (true inverse; singular -> "U(i, i) is zero.").
 * replaces pr.cu:547-570 (pb.rs:36-41). */
const char* q1gate_inv(qdc_complex* state, const qdc_complex* gate, size_t pos,
                       size_t qubits_number);

/* Two-qubit gate, row-major 4x4, pos2 = most significant local index bit:
 * out[2Q2+Q1] = sum U[8Q2+4Q1+2P2+P1] in[P2,P1].
 * replaces pr.cu:573-620 (pb.rs:42-48). */
const char* q2gate(qdc_complex* state, const qdc_complex* gate, size_t pos2,
                   size_t pos1, size_t qubits_number);

/* psi <- U^-1 psi for a 4x4 U.  replaces pr.cu:622-646 (pb.rs:49-55). */
const char* q2gate_inv(qdc_complex* state, const qdc_complex* gate, size_t pos2,
                       size_t pos1, size_t qubits_number);

/* Diagonal two-qubit gate: psi[i] *= d[2 bit(i,pos2) + bit(i,pos1)].
 * replaces pr.cu:649-686 (pb.rs:56-62). */
const char* q2gate_diag(qdc_complex* state, const qdc_complex* gate, size_t pos2,
                        size_t pos1, size_t qubits_number);

/* rho[2p+q] += sum psi[p] conj(psi[q]).  replaces pr.cu:689-776 (pb.rs:68-73). */
const char* get_q1density(const qdc_complex* state, qdc_complex* density, size_t pos,
                          size_t qubits_number);

/* rho[8p2+4p1+2q2+q1] += sum psi[p2,p1] conj(psi[q2,q1]).
 * replaces pr.cu:779-876 (pb.rs:74-80). */
const char* get_q2density(const qdc_complex* state, qdc_complex* density, size_t pos2,
                          size_t pos1, size_t qubits_number);

/* G[2p+q] += sum bwd[p] fwd[q] (no conjugation).  replaces pr.cu:202-292 (pb.rs:81-87). */
const char* q1grad(const qdc_complex* fwd, const qdc_complex* bwd, qdc_complex* grad,
                   size_t pos, size_t qubits_number);

/* G[8p2+4p1+2q2+q1] += sum bwd[p2,p1] fwd[q2,q1].  replaces pr.cu:295-395 (pb.rs:88-95). */
const char* q2grad(const qdc_complex* fwd, const qdc_complex* bwd, qdc_complex* grad,
                   size_t pos2, size_t pos1, size_t qubits_number);

/* G[2p+q] += sum_{i: bit(i,pos2)=p, bit(i,pos1)=q} bwd[i] fwd[i].
 * replaces pr.cu:398-493 (pb.rs:96-103). */
const char* q2grad_diag(const qdc_complex* fwd, const qdc_complex* bwd, qdc_complex* grad,
                        size_t pos2, size_t pos1, size_t qubits_number);

/* dst = 2 conj(src).  replaces pr.cu:904-929 (pb.rs:104-108). */
void conj_and_double(const qdc_complex* src, qdc_complex* dst, size_t qubits_number);

/* dst += src.  replaces pr.cu:931-953 (pb.rs:109-113). */
void add(const qdc_complex* src, qdc_complex* dst, size_t qubits_number);

/* dst = src.  replaces pr.cu:879-901 (pb.rs:114-118). */
void copy(const qdc_complex* src, qdc_complex* dst, size_t qubits_number);

#ifdef __cplusplus
}
#endif

#endif /* QDC_PRIMITIVES_H */
