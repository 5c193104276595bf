/*
 * cpu_ref.c — C/OpenMP restatement of the reference's CUDA primitives
 * (src/primitives.cu:176-953) on host memory.  TEST INFRASTRUCTURE ONLY: it is the
 * independent checker for the HIP kernels (tests/) and the CPU baseline timed by bench.py
 * ("cpu_baseline", kind "port").  The product library never links it.
 *
 * Index rules follow the CUDA kernels line by line:
 *   INSERT_ZERO(mask, off) = ((mask & off) << 1) | (~mask & off)      primitives.cu:104-105
 *   two-qubit kernels insert the zero at the lower position first      primitives.cu:305-321
 * but with 64-bit sizes (the reference's `1 << n` is an int, primitives.cu:147).
 * Reductions follow the reference's 128 x 128-thread summation order and accumulate `+=` into
 * the caller's buffer like the host loops of primitives.cu:281-288.  Arithmetic is sequential
 * per element: out[p] = sum_q g[2p+q] in[q].
 *
 * Build: gcc -O3 -fopenmp -shared -fPIC [-DQDC_F64]  (oracle/Makefile)
 */
#include <complex.h>
#include <omp.h>
#include <stddef.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef QDC_F64
typedef double complex C;
typedef double R;
#define CONJ conj
#else
typedef float complex C;
typedef float R;
#define CONJ conjf
#endif

#define EXPORT __attribute__((visibility("default")))

static inline uint64_t insert_zero(uint64_t mask, uint64_t off) {
  return ((mask & off) << 1) | (~mask & off);
}

/* primitives.cu:513-532 */
EXPORT void cref_q1gate(C* s, const C* g, size_t pos, size_t n) {
  const uint64_t mask = UINT64_MAX << pos, stride = (uint64_t)1 << pos;
  const int64_t batch = (int64_t)(((uint64_t)1 << n) >> 1);
#pragma omp parallel for schedule(static)
  for (int64_t tid = 0; tid < batch; ++tid) {
    const uint64_t b = insert_zero(mask, (uint64_t)tid);
    const C x0 = s[b], x1 = s[b + stride];
    s[b] = g[0] * x0 + g[1] * x1;
    s[b + stride] = g[2] * x0 + g[3] * x1;
  }
}

static inline void q2_masks(size_t pos2, size_t pos1, uint64_t* min_mask, uint64_t* max_mask) {
  const uint64_t m1 = UINT64_MAX << pos1, m2 = UINT64_MAX << pos2;
  *max_mask = m1 < m2 ? m1 : m2; /* MIN(mask1, mask2): the higher position */
  *min_mask = m1 < m2 ? m2 : m1; /* MAX(mask1, mask2): the lower position */
}

/* primitives.cu:573-606 */
EXPORT void cref_q2gate(C* s, const C* g, size_t pos2, size_t pos1, size_t n) {
  uint64_t mn, mx;
  q2_masks(pos2, pos1, &mn, &mx);
  const uint64_t s1 = (uint64_t)1 << pos1, s2 = (uint64_t)1 << pos2;
  const int64_t batch = (int64_t)(((uint64_t)1 << n) >> 2);
#pragma omp parallel for schedule(static)
  for (int64_t tid = 0; tid < batch; ++tid) {
    const uint64_t b = insert_zero(mx, insert_zero(mn, (uint64_t)tid));
    C in[4], out[4];
    for (int p2 = 0; p2 < 2; ++p2)
      for (int p1 = 0; p1 < 2; ++p1) in[2 * p2 + p1] = s[b + p2 * s2 + p1 * s1];
    for (int q = 0; q < 4; ++q) {
      C t = 0;
      for (int p = 0; p < 4; ++p) t += g[4 * q + p] * in[p];
      out[q] = t;
    }
    s[b] = out[0];
    s[b + s1] = out[1];
    s[b + s2] = out[2];
    s[b + s1 + s2] = out[3];
  }
}

/* primitives.cu:649-672 */
EXPORT void cref_q2gate_diag(C* s, const C* d, size_t pos2, size_t pos1, size_t n) {
  uint64_t mn, mx;
  q2_masks(pos2, pos1, &mn, &mx);
  const uint64_t s1 = (uint64_t)1 << pos1, s2 = (uint64_t)1 << pos2;
  const int64_t batch = (int64_t)(((uint64_t)1 << n) >> 2);
#pragma omp parallel for schedule(static)
  for (int64_t tid = 0; tid < batch; ++tid) {
    const uint64_t b = insert_zero(mx, insert_zero(mn, (uint64_t)tid));
    s[b] *= d[0];
    s[b + s1] *= d[1];
    s[b + s2] *= d[2];
    s[b + s1 + s2] *= d[3];
  }
}

/* Reductions, in the reference's summation order (primitives.cu:202-292 and its siblings):
 * BLOCKS_NUM x THREADS_NUM = 128 x 128 CUDA threads (pr.cu:6-7); thread v accumulates the items
 * tid = v, v + 16384, v + 2 * 16384, ... sequentially (PARALLEL_FOR, pr.cu:72-80); each block
 * folds its 128 partials by the shared-memory tree s = 64, 32, ..., 1 (cache[t] += cache[t + s]);
 * the host then adds the 128 block sums in block order into the caller's buffer with `+=`
 * (pr.cu:281-288).  So the f32 rounding of a long reduction is the reference's, not that of one
 * long sequential sum per OpenMP thread (which at n = 24 is ~1e-4 in f32, 100x the reference's).
 * Items are visited row by row (row r = items r * 16384 .. + 16383) so memory streams in order;
 * an OpenMP thread owns a range of virtual threads and their K accumulators. */
#define REF_BLOCKS 128
#define REF_THREADS 128
#define REF_VT (REF_BLOCKS * REF_THREADS)
#define REDUCE_BEGIN(K, BATCH)                                                   \
  enum { K_ = (K) };                                                             \
  const int64_t batch_ = (int64_t)(BATCH);                                       \
  C* part_ = (C*)calloc((size_t)REF_VT * K_, sizeof(C));                         \
  if (!part_) abort();                                                           \
  _Pragma("omp parallel")                                                        \
  {                                                                              \
    const int nt_ = omp_get_num_threads(), me_ = omp_get_thread_num();           \
    const int64_t v0_ = (int64_t)REF_VT * me_ / nt_, v1_ = (int64_t)REF_VT * (me_ + 1) / nt_; \
    for (int64_t r0_ = 0; r0_ < batch_; r0_ += REF_VT)                           \
      for (int64_t v_ = v0_; v_ < v1_ && r0_ + v_ < batch_; ++v_) {              \
        const int64_t tid = r0_ + v_;                                            \
        C* acc = part_ + (size_t)v_ * K_;
#define REDUCE_END(out)                                                          \
      }                                                                          \
  }                                                                              \
  for (int b_ = 0; b_ < REF_BLOCKS; ++b_) {                                      \
    C* blk_ = part_ + (size_t)b_ * REF_THREADS * K_;                             \
    for (int s_ = REF_THREADS / 2; s_ != 0; s_ /= 2)                             \
      for (int t_ = 0; t_ < s_; ++t_)                                            \
        for (int k_ = 0; k_ < K_; ++k_) blk_[t_ * K_ + k_] += blk_[(t_ + s_) * K_ + k_]; \
  }                                                                              \
  for (int b_ = 0; b_ < REF_BLOCKS; ++b_)                                        \
    for (int k_ = 0; k_ < K_; ++k_) (out)[k_] += part_[(size_t)b_ * REF_THREADS * K_ + k_]; \
  free(part_);

/* primitives.cu:689-739 */
EXPORT void cref_q1density(const C* s, C* rho, size_t pos, size_t n) {
  const uint64_t mask = UINT64_MAX << pos, stride = (uint64_t)1 << pos;
  REDUCE_BEGIN(4, ((uint64_t)1 << n) >> 1)
    const uint64_t b = insert_zero(mask, (uint64_t)tid);
    for (int q = 0; q < 2; ++q)
      for (int p = 0; p < 2; ++p) acc[2 * p + q] += s[p * stride + b] * CONJ(s[q * stride + b]);
  REDUCE_END(rho)
}

/* primitives.cu:779-837 */
EXPORT void cref_q2density(const C* s, C* rho, size_t pos2, size_t pos1, size_t n) {
  uint64_t mn, mx;
  q2_masks(pos2, pos1, &mn, &mx);
  const uint64_t s1 = (uint64_t)1 << pos1, s2 = (uint64_t)1 << pos2;
  REDUCE_BEGIN(16, ((uint64_t)1 << n) >> 2)
    const uint64_t b = insert_zero(mx, insert_zero(mn, (uint64_t)tid));
    C x[4];
    for (int p2 = 0; p2 < 2; ++p2)
      for (int p1 = 0; p1 < 2; ++p1) x[2 * p2 + p1] = s[b + p2 * s2 + p1 * s1];
    for (int p = 0; p < 4; ++p)
      for (int q = 0; q < 4; ++q) acc[4 * p + q] += x[p] * CONJ(x[q]);
  REDUCE_END(rho)
}

/* primitives.cu:202-253 */
EXPORT void cref_q1grad(const C* f, const C* bw, C* grad, size_t pos, size_t n) {
  const uint64_t mask = UINT64_MAX << pos, stride = (uint64_t)1 << pos;
  REDUCE_BEGIN(4, ((uint64_t)1 << n) >> 1)
    const uint64_t b = insert_zero(mask, (uint64_t)tid);
    for (int q = 0; q < 2; ++q)
      for (int p = 0; p < 2; ++p) acc[2 * p + q] += bw[p * stride + b] * f[q * stride + b];
  REDUCE_END(grad)
}

/* primitives.cu:295-354 */
EXPORT void cref_q2grad(const C* f, const C* bw, C* grad, size_t pos2, size_t pos1, size_t n) {
  uint64_t mn, mx;
  q2_masks(pos2, pos1, &mn, &mx);
  const uint64_t s1 = (uint64_t)1 << pos1, s2 = (uint64_t)1 << pos2;
  REDUCE_BEGIN(16, ((uint64_t)1 << n) >> 2)
    const uint64_t b = insert_zero(mx, insert_zero(mn, (uint64_t)tid));
    C xf[4], xb[4];
    for (int p2 = 0; p2 < 2; ++p2)
      for (int p1 = 0; p1 < 2; ++p1) {
        xf[2 * p2 + p1] = f[b + p2 * s2 + p1 * s1];
        xb[2 * p2 + p1] = bw[b + p2 * s2 + p1 * s1];
      }
    for (int p = 0; p < 4; ++p)
      for (int q = 0; q < 4; ++q) acc[4 * p + q] += xb[p] * xf[q];
  REDUCE_END(grad)
}

/* primitives.cu:398-452 */
EXPORT void cref_q2grad_diag(const C* f, const C* bw, C* grad, size_t pos2, size_t pos1,
                             size_t n) {
  uint64_t mn, mx;
  q2_masks(pos2, pos1, &mn, &mx);
  const uint64_t s1 = (uint64_t)1 << pos1, s2 = (uint64_t)1 << pos2;
  REDUCE_BEGIN(4, ((uint64_t)1 << n) >> 2)
    const uint64_t b = insert_zero(mx, insert_zero(mn, (uint64_t)tid));
    for (int q = 0; q < 2; ++q)
      for (int p = 0; p < 2; ++p)
        acc[2 * p + q] += bw[p * s2 + q * s1 + b] * f[p * s2 + q * s1 + b];
  REDUCE_END(grad)
}

/* primitives.cu:176-187 */
EXPORT void cref_set2standard(C* s, size_t n) {
  const int64_t size = (int64_t)((uint64_t)1 << n);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < size; ++i) s[i] = 0;
  s[0] = 1;
}

/* primitives.cu:879-887 */
EXPORT void cref_copy(const C* src, C* dst, size_t n) {
  const int64_t size = (int64_t)((uint64_t)1 << n);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < size; ++i) dst[i] = src[i];
}

/* primitives.cu:904-915 */
EXPORT void cref_conj_and_double(const C* src, C* dst, size_t n) {
  const int64_t size = (int64_t)((uint64_t)1 << n);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < size; ++i) dst[i] = 2 * CONJ(src[i]);
}

/* primitives.cu:931-939 */
EXPORT void cref_add(const C* src, C* dst, size_t n) {
  const int64_t size = (int64_t)((uint64_t)1 << n);
#pragma omp parallel for schedule(static)
  for (int64_t i = 0; i < size; ++i) dst[i] += src[i];
}

EXPORT int cref_threads(void) {
  int t = 1;
#pragma omp parallel
  {
#pragma omp single
    t = omp_get_num_threads();
  }
  return t;
}

/* thread count of the following calls (bench.py times the baseline at 1 thread and at all) */
EXPORT void cref_set_threads(int t) { omp_set_num_threads(t > 0 ? t : 1); }
