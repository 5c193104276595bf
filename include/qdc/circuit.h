/*
 * qdc/circuit.h — native circuit interpreter over the HIP hot path.
 *
 * The reference implements this layer in Rust: `QuantizedTensor` (src/quantized_tensor.rs:
 * 54-238) and the PyO3 class `Circuit` (src/circuit.rs:86-430).  Rust is not available on
 * this platform, so the same semantics are provided by a C++ runtime behind this C ABI;
 * the Python class `quantum_differentiable_circuit.Circuit` is a thin ctypes shim over it
 * (see INTEGRATION.md for the equivalent Rust/cgo/ctypes bindings).
 *
 * Semantics follow circuit.rs exactly (instruction list, FIFO gate consumption, densities
 * in instruction order, the O(1)-memory reverse sweep, zero gradients for variable gates
 * met before any density cotangent, the panic messages).  What differs is only HOW it is
 * executed: the reverse sweep is fused (uncompute + gradient + cotangent pull-back in one
 * HBM pass), density cotangents are injected without a temporary state, and all gradients
 * and densities stay on the device until one copy at the end of the call.
 *
 * Gates are passed flattened: `gates` = concatenation of every gate buffer, `lens[i]` = the
 * number of complex entries of gate i.  Error convention as in primitives.h.
 */
#ifndef QDC_CIRCUIT_H
#define QDC_CIRCUIT_H

#include <stddef.h>

#include "qdc/primitives.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Instruction kinds, in the order of `enum Instruction` (src/circuit.rs:53-68). */
enum qdc_kind {
  QDC_CONST_Q2 = 0,
  QDC_VAR_Q2 = 1,
  QDC_CONST_Q2_NONU = 2,
  QDC_VAR_Q2_NONU = 3,
  QDC_CONST_Q2_DIAG = 4,
  QDC_VAR_Q2_DIAG = 5,
  QDC_CONST_Q1 = 6,
  QDC_CONST_Q1_NONU = 7,
  QDC_VAR_Q1 = 8,
  QDC_VAR_Q1_NONU = 9,
  QDC_Q2_DENSITY = 10,
  QDC_Q1_DENSITY = 11,
  QDC_DIFF_Q2_DENSITY = 12,
  QDC_DIFF_Q1_DENSITY = 13
};

/* Execution modes of qdc_circuit_execute: Circuit::run (circuit.rs:164-212) returns every
 * density; Circuit::forward (circuit.rs:214-264) only the Diff* ones. */
enum qdc_mode { QDC_MODE_RUN = 0, QDC_MODE_FORWARD = 1 };

typedef struct qdc_circuit qdc_circuit;

/* Circuit::new (circuit.rs:95-103): initial state |0...0>, on the current HIP device. */
const char* qdc_circuit_new(qdc_circuit** out, size_t qubits_number);
void qdc_circuit_free(qdc_circuit* c);
size_t qdc_circuit_qubits(const qdc_circuit* c);

/* Circuit::set_state_from_vector (circuit.rs:104-106 → quantized_tensor.rs:76-80). */
const char* qdc_circuit_set_state_from_vector(qdc_circuit* c, const qdc_complex* vec,
                                              size_t len);

/* Circuit::add_* / get_*_dens_op* (circuit.rs:108-162).  For one-qubit kinds pass the
 * position as `pos2` (pos1 is ignored). */
const char* qdc_circuit_push(qdc_circuit* c, int kind, size_t pos2, size_t pos1);
size_t qdc_circuit_len(const qdc_circuit* c);

/* Number of complex values written to `densities` by qdc_circuit_execute(mode): 4 per
 * one-qubit and 16 per two-qubit density, in instruction order. */
size_t qdc_circuit_output_size(const qdc_circuit* c, int mode);
/* Number of complex values written to `grads` by qdc_circuit_backward: 4 / 16 / 4 per
 * Q1 / Q2 / Q2Diag variable gate, in forward order. */
size_t qdc_circuit_grad_size(const qdc_circuit* c);

/* Circuit::run / Circuit::forward. */
const char* qdc_circuit_execute(qdc_circuit* c, int mode, const qdc_complex* const_gates,
                                const size_t* const_lens, size_t n_const,
                                const qdc_complex* var_gates, const size_t* var_lens,
                                size_t n_var, qdc_complex* densities);

/* Circuit::backward (circuit.rs:266-429).  `dens_grads` are the (already conjugated,
 * circuit.py:193) cotangents of the Diff* densities, 4 or 16 entries each, forward order. */
const char* qdc_circuit_backward(qdc_circuit* c, const qdc_complex* dens_grads,
                                 const size_t* dens_lens, size_t n_dens,
                                 const qdc_complex* const_gates, const size_t* const_lens,
                                 size_t n_const, const qdc_complex* var_gates,
                                 const size_t* var_lens, size_t n_var, qdc_complex* grads);

/* Copies of the device states, for tests and debugging (QuantizedTensor::get_cpu_state_copy,
 * quantized_tensor.rs:91-99).  which: 0 = current (fwd) state, 1 = initial state,
 * 2 = backward state (after a backward call).  Always in logical qubit order (fused passes
 * may keep fwd / bwd in a permuted layout on the device: qdc_circuit_layout). */
const char* qdc_circuit_get_state(qdc_circuit* c, int which, qdc_complex* host, size_t len);

/* Wait for all work queued by this circuit. */
const char* qdc_circuit_sync(qdc_circuit* c);

/* ---- measurement ------------------------------------------------------------------- */
typedef struct qdc_kernel_stat {
  char name[32];
  size_t launches;
  double total_ms;    /* sum of HIP-event durations of this kernel's launches */
  double algo_bytes;  /* sum of algorithmic HBM bytes (SURVEY.md §8 d) */
  double algo_flops;  /* sum of algorithmic real FLOPs (fused passes; 0 for streaming kernels) */
} qdc_kernel_stat;

/* Bracket every launch of this circuit's stream with HIP events (on = 1) or stop (0);
 * enabling clears previously collected records. */
const char* qdc_circuit_profile(qdc_circuit* c, int on);
/* Synchronise and aggregate the records per kernel name; returns the number of kernels
 * (writes at most `cap` entries). */
size_t qdc_circuit_profile_collect(qdc_circuit* c, qdc_kernel_stat* out, size_t cap);
/* Host time of the circuit's calls since the last reset (reset = 1 clears after reading):
 * out[0..5] run / forward, out[6..11] backward, each (calls, setup ms, schedule ms, program
 * build ms, launch ms, finish ms: stream sync, result copies, gradient reconstruction).
 * Returns the number of values written (at most n, at most 12). */
size_t qdc_circuit_host_times(qdc_circuit* c, double* out, size_t n, int reset);

/* Library build information: "f32"/"f64", offload arch. */
const char* qdc_build_info(void);

/* ---- sharded state (no reference counterpart) -------------------------
 * The 2^n state splits over G = 2^g ranks by its high (physical) qubits.  A qubit map tracks
 * which logical qubit sits at which physical bit; an op that needs a global qubit is preceded
 * by a REMAP: one all-to-all per state that swaps all g global qubits with g local ones.
 * Densities and gradients are summed over ranks (one all-reduce per call), so every rank
 * returns the full results.  Transports:
 *   - qdc_circuit_new_sharded: one shard per process, RCCL over xGMI (qdc_comm_*);
 *   - qdc_circuit_new_devices: one process, one shard per GPU, RCCL (ncclCommInitAll);
 *   - qdc_circuit_new_local_shards: every shard on the current GPU, exchanged with device
 *     copies (the same data path on one GPU; used by the single-GPU parity tests). */
typedef struct qdc_comm qdc_comm;
/* rank 0 creates the id and ships it to the other ranks (quantum_differentiable_circuit.
 * distributed: through a per-launch file, no second collective stack) */
const char* qdc_comm_unique_id(unsigned char id[128]);
/* collective over all ranks; uses the current HIP device */
const char* qdc_comm_init(qdc_comm** out, int rank, int world, const unsigned char id[128]);
void qdc_comm_free(qdc_comm* comm);
/* Collective: sum (op 0) or maximum (op 1) of `count` <= 64 host doubles over the ranks, in
 * place on every rank; count 0 is a barrier.  Returns after the result is on the host. */
const char* qdc_comm_allreduce(qdc_comm* comm, double* vals, int count, int op);

const char* qdc_circuit_new_sharded(qdc_circuit** out, size_t qubits_number, qdc_comm* comm);
const char* qdc_circuit_new_local_shards(qdc_circuit** out, size_t qubits_number, int shards);
/* One process driving one shard per listed device (ndev a power of two): distinct devices
 * communicate through RCCL communicators made by ncclCommInitAll (collectives grouped over the
 * shards' streams); the same device repeated keeps every shard on it, each on its own stream,
 * exchanged by device copies ordered with events. */
const char* qdc_circuit_new_devices(qdc_circuit** out, size_t qubits_number, int ndev,
                                    const int* devices);

/* Current layout of the forward state: phys[q] = physical bit of logical qubit q (n entries),
 * plus world size, this process's first rank and its number of local shards. */
const char* qdc_circuit_layout(const qdc_circuit* c, unsigned* phys, int* world, int* rank,
                               int* local_shards);
/* Copy of one local shard (2^(n-g) amplitudes, physical order). which: 0 fwd, 1 initial, 2 bwd */
const char* qdc_circuit_get_shard(qdc_circuit* c, int which, int shard, qdc_complex* host,
                                  size_t len);

/* Collective over the circuit's communicator: the whole state (2^n amplitudes, PHYSICAL
 * order: shard r = physical index bits above n - g equal to r) on every process, shards of
 * other processes broadcast through one shard of device staging.  which: as qdc_circuit_get_shard */
const char* qdc_circuit_gather_state(qdc_circuit* c, int which, qdc_complex* host, size_t len);

/* A range [offset, offset + len) of one local shard in PHYSICAL order (qubits may be permuted:
 * qdc_circuit_layout); for streaming reads of states too large for one host copy. */
const char* qdc_circuit_get_range(qdc_circuit* c, int which, int shard, size_t offset,
                                  qdc_complex* host, size_t len);

/* ---- the sharding planner (host only, no GPU) ---------------------------------------- */
/* QDC_PLAN_FORWARD_MIRROR: a forward whose plan, run in reverse with every remap undone, is the
 * backward's (mirrored reverse sweeps): ops keep the order relations of both directions. */
enum qdc_plan_mode {
  QDC_PLAN_RUN = 0,
  QDC_PLAN_FORWARD = 1,
  QDC_PLAN_BACKWARD = 2,
  QDC_PLAN_FORWARD_MIRROR = 3
};
enum qdc_plan_type { QDC_PLAN_OP = 0, QDC_PLAN_REMAP = 1 };
typedef struct qdc_plan_op {
  int type;             /* QDC_PLAN_OP: run instruction `instr` at physical (pos2, pos1) */
  int instr;            /* QDC_PLAN_REMAP: all-to-all with these local victims -> rank bits */
  unsigned pos2, pos1;
  unsigned victims[8];  /* ascending; victim j becomes rank bit j */
  unsigned nvictims;
  int pack;             /* victims are not the top local bits: pack before the all-to-all */
} qdc_plan_op;
/* Plan one pass of `count` instructions over `world` ranks, starting from `start_phys`
 * (NULL = identity).  Writes at most `cap` ops, returns the total; `end_phys` (nullable)
 * receives the final layout. */
size_t qdc_plan(size_t qubits_number, size_t world, const int* kinds, const unsigned* pos2,
                const unsigned* pos1, size_t count, int mode, const unsigned* start_phys,
                qdc_plan_op* out, size_t cap, unsigned* end_phys);

/* ---- Fused-pass schedule ----------------------------------------------
 * The runtime's own scheduler, exposed for tests and tools: which plan ops share an HBM pass
 * and in which order they run.  kinds[n_instr]: instruction kinds; inexact[n_instr]
 * (nullable = all 0): 1 marks a gate whose matrix is not unitary to working precision;
 * plan[n_plan]: from qdc_plan; first_inject: plan index of the first cotangent injection
 * (backward; SIZE_MAX otherwise); lcmin / max_ops: tile rows and pass size (<= 0: defaults).
 * Outputs, per item in execution order: item_info[12*i ..] = {type (0 single op, 1 remap,
 * 2 fused pass), stages, lc, h, hb[0..7]}; stage_len[]: ops per stage, flattened over items;
 * op_order[]: plan indices in execution order.  Returns the number of items, or SIZE_MAX if an
 * output capacity is too small. */
size_t qdc_fusion_schedule(size_t local_qubits, int backward, size_t first_inject,
                           const int* kinds, const unsigned char* inexact, size_t n_instr,
                           const qdc_plan_op* plan, size_t n_plan, int lcmin, int max_ops,
                           unsigned* item_info, size_t item_cap, unsigned* stage_len,
                           size_t stage_cap, unsigned* op_order, size_t op_cap);

/* Test hook (host only): the register-layout plan of a register-resident pass (qdc_rq.hpp)
 * over n stages with kinds[] (0 one-qubit, 1 two-qubit, 2 diagonal) on tile bits t1[], t2[]
 * (t1 < t2; one-qubit: t1 == t2) of a tile with tile_bits amplitude bits, on layouts of
 * `slots` (4 or 5) register slots; deps[i] = bit mask of the earlier stages stage i must
 * follow (NULL: none).  steps[8*i..]: {type (2 load layout, 1 relayout, 0 stage, 3 store
 * layout), stage index, slot case (two-qubit: 8 * slot(t1) + slot(t2); one-qubit: slot),
 * layout slots 0..4 (~0 past `slots`)}, the load layout first and the store layout last.
 * Returns the number of steps, or SIZE_MAX if cap is too small or the arguments are invalid. */
size_t qdc_rq_plan(unsigned tile_bits, unsigned slots, const unsigned* kinds, const unsigned* t1,
                   const unsigned* t2, const unsigned long long* deps, size_t n,
                   unsigned* steps, size_t cap);

/* Test hook (host only): the specialized kernel of a pass over n stages (kinds / t1 / t2 / deps
 * as qdc_rq_plan) — f32 tile_bits 11: a five-slot two-state reverse pass, every stage
 * accumulating Gamma; 12: a four-slot one-state forward pass; f64: 10 two-state, 11 one-state: the
 * runtime's source generator and hipcc for gfx950, as a circuit call on a GPU box runs them
 * (qdc_jit.hpp), without loading the code object.  name_out (cap >= 128) receives the kernel
 * name, a NUL, then the code object's path.  Returns NULL, or an error message. */
const char* qdc_spec_selftest(unsigned tile_bits, const unsigned* kinds, const unsigned* t1,
                              const unsigned* t2, const unsigned long long* deps, size_t n,
                              char* name_out, size_t cap);
/* Test hook (host only): as qdc_spec_selftest for nprog pass programs at once (counts[p] stages
 * each, the stage arrays concatenated), compiled in one call of the cache (as a circuit call
 * compiles its missing kernels together).  names_out receives the kernel names, each NUL-ended. */
const char* qdc_spec_selftest_batch(unsigned tile_bits, const size_t* counts, size_t nprog,
                                    const unsigned* kinds, const unsigned* t1, const unsigned* t2,
                                    const unsigned long long* deps, char* names_out, size_t cap);

/* Test hook (host only): the launch geometry a single-gate op gets (qdc_device.hpp plan_gate)
 * on an n-qubit state: R = 2 (one-qubit, pos2 == pos1) or 4; two_states: the op reads both
 * states (tile of 2^9 chunks, else 2^10); far_tile: targets beyond chunk bit 5 go to the tile
 * family as row bits too (QDC_TILE_FAR).  out[0..9] = {tile, mode (direct), l, h, hb0, hb1,
 * t1, t2, ntiles (tile) or items (direct) low 32 bits, high 32 bits}.  Returns 0, or -1 on
 * invalid arguments. */
int qdc_gate_plan(unsigned n, unsigned R, unsigned pos2, unsigned pos1, int two_states,
                  int far_tile, unsigned* out);

/* Test hook (host only): the LANE family's geometry (qdc_device.hpp plan_lane; one chunk per
 * lane, partner amplitudes across lanes).  out[0..9] = {in-chunk gate bit + 1 (0: none),
 * contiguous low chunk bits of a 64-chunk unit, far targets, their chunk bits f0 and f1,
 * lane masks of gate bits 0 (pos1) and 1 (pos2), units low 32 bits, high 32 bits, units per
 * wave (reduces bit 0: a grid of about 2048 blocks)}; reduces bit 1: the block-wide variant
 * (k_lane_blk: 1024-chunk units, thread masks).  Returns 0, 1 when the state has fewer chunks
 * than a unit, -1 on invalid arguments. */
int qdc_lane_plan(unsigned n, unsigned R, unsigned pos2, unsigned pos1, int reduces,
                  unsigned* out);

/* The specialized-kernel cache of this process (qdc_jit.hpp).  stats[0..8] (up to n) =
 * {kernels compiled by this process, kernels waited for while another process compiled them,
 * (kernel, device) loads, seconds compiling, seconds waiting, seconds in the cache overall
 * (compile + wait + load), 1 if specialization is on else 0, launches of specialized kernels,
 * kernels queued for the background compiler}.  Returns the values written. */
size_t qdc_jit_stats(double* stats, size_t n);

/* Wait up to timeout_s seconds for the background compiler (programs with more distinct
 * specialized kernels than QDC_SPEC_MAX compile there while generic kernels run their passes)
 * to drain its queue.  Returns the kernels still queued. */
size_t qdc_jit_wait(double timeout_s);

/* The cache directory in use (dir_out, cap >= 2): NULL, or an error message when
 * specialization is off (no hipcc, kernel headers changed since the build, no private
 * directory). */
const char* qdc_jit_dir(char* dir_out, size_t cap);

/* Test hook (host only): the build fingerprint a library with the given -D switches (NULL: this
 * library's own), compiler identity text and kernel headers (the .hpp files of csrc_dir plus
 * the .h files of csrc_dir/../../include/qdc) would name its kernels with (qdc_jit.hpp), and
 * the header hash alone.  Returns NULL, or an error message. */
const char* qdc_spec_fingerprint(const char* defines, const char* compiler, const char* csrc_dir,
                                 unsigned long long* fingerprint, unsigned long long* source_hash);

/* Ahead-of-time compilation (host only, no GPU; build time): a dry run of forward(cg, vg) then
 * backward(dg, cg, vg) on a circuit of `count` instructions (kinds[], pos2[], pos1[] as
 * qdc_circuit_push) over `world` shards builds the runtime's own pass programs and compiles
 * every specialized kernel they would launch into the cache directory (QDC_JIT_DIR).  The
 * runtime then finds them there, or in the read-only prebuilt directory next to the library
 * (<pkg>/jit-prebuilt, QDC_JIT_PREBUILT).  *kernels (nullable): the distinct kernels.  Returns
 * NULL, or an error message. */
const char* qdc_precompile(size_t qubits_number, int world, const int* kinds,
                           const unsigned* pos2, const unsigned* pos1, size_t count,
                           const qdc_complex* const_gates, const size_t* const_lens, size_t n_const,
                           const qdc_complex* var_gates, const size_t* var_lens, size_t n_var,
                           const qdc_complex* dens_grads, const size_t* dens_lens, size_t n_dens,
                           size_t* kernels);

/* Test hook (host only): the runtime's forward schedule of `count` instructions over `world`
 * shards, replayed against its layout: every op's positions where its logical qubits are,
 * every remap's victims local and ascending (permuting passes relabel later remaps).  *items /
 * *swaps (nullable): the schedule's items and permuting swaps.  Returns NULL, or the first
 * inconsistency. */
const char* qdc_check_schedule(size_t qubits_number, int world, const int* kinds,
                               const unsigned* pos2, const unsigned* pos1, size_t count,
                               size_t* items, size_t* swaps);

/* One matrix a call applies to the forward state (qdc_trace_program): dir 0 forward, 1 the
 * backward's uncompute; its logical qubits q2, q1 (row index 2 bit(q2) + bit(q1); q2 == q1 and
 * R == 2 for one qubit); m: the R x R row-major matrix as the kernels apply it (working precision,
 * diagonals expanded); mirrored: the exact adjoint of the forward's recorded stage matrix;
 * single: a single-gate item, else a fused stage; item: its pass in the call's schedule. */
typedef struct qdc_trace_op {
  unsigned dir, item, q2, q1, R, diag, mirrored, single;
  qdc_complex m[16];
} qdc_trace_op;

/* Test hook (host only, the drift emulator tools/drift_emu.py): a dry run of forward(cg, vg)
 * then backward(dg, cg, vg) as qdc_precompile, returning every matrix the two calls apply to the
 * forward state, in order, into out[0..cap).  *count: the number of matrices (when > cap, call
 * again with a larger buffer).  Returns NULL, or an error message. */
const char* qdc_trace_program(size_t qubits_number, int world, const int* kinds,
                              const unsigned* pos2, const unsigned* pos1, size_t count,
                              const qdc_complex* const_gates, const size_t* const_lens,
                              size_t n_const, const qdc_complex* var_gates,
                              const size_t* var_lens, size_t n_var, const qdc_complex* dens_grads,
                              const size_t* dens_lens, size_t n_dens, qdc_trace_op* out, size_t cap,
                              size_t* n_out);

#ifdef __cplusplus
}
#endif

#endif /* QDC_CIRCUIT_H */
