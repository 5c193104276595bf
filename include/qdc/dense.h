/*
 * qdc/dense.h — extensions of the C ABI beyond the reference's 18 entry points
 * (include/qdc/primitives.h).  Same conventions: a state is a device buffer of 2^n
 * interleaved {re, im} amplitudes, gate pointers are HOST memory read before the call
 * returns, NULL = success, otherwise a library-owned message.
 *
 * Dense k-qubit gates are SURVEY.md §8 f rank 4: the reference stops at 2-qubit gates
 * (src/primitives.cu:513-686); a user wanting a 3..5-qubit unitary there must decompose it.
 * Here k >= 3 runs on the matrix cores (csrc/qdc_qk.hpp: v_mfma_{f32,f64}_16x16x4 with the
 * gate resident in VGPRs), k = 1, 2 on the q1gate / q2gate kernels.
 */
#ifndef QDC_DENSE_H
#define QDC_DENSE_H

#include <stddef.h>

#include "qdc/circuit.h"
#include "qdc/primitives.h"

#ifdef __cplusplus
extern "C" {
#endif

/* state <- (U on qubits pos[0..k)) state, 1 <= k <= 5, positions distinct and < n.
 * gate: 2^k x 2^k complex, row-major; local index bit (k-1-b) is qubit pos[b] (pos[0] is
 * the most significant, as q2gate's pos2).  Errors as q2gate ("pos is out of the bound.",
 * "positions must be different."). */
const char* qdc_qkgate(qdc_complex* state, const qdc_complex* gate, const size_t* pos, size_t k,
                       size_t n);

/* The primitives' stream (every entry point above is ordered on it): wait for it. */
const char* qdc_abi_sync(void);

/* Per-launch HIP-event profiling of the primitives' stream (as qdc_circuit_profile):
 * on != 0 resets and starts, 0 stops; collect returns per-kernel sums. */
const char* qdc_abi_profile(int on);
size_t qdc_abi_profile_collect(qdc_kernel_stat* out, size_t cap);

#ifdef __cplusplus
}
#endif

#endif /* QDC_DENSE_H */
