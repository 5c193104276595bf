// qdc_jit.hpp — the specialized pass kernels (qdc_spec.hpp; two-state reverse passes and
// one-state forward passes): source per pass program, compiled with hipcc for gfx950 on first
// use, cached on disk and per device.
//
// A pass program becomes a functor of straight-line stage calls.  Its kernel is named by the
// hash of its source and of the build fingerprint (the library's -D switches, hipcc's path and
// --version text, the compile options, and the bytes of every kernel header), so passes with
// the same program share one kernel across circuits and processes, and no two builds ever share
// one.  Code objects live in a private cache directory (QDC_JIT_DIR, else $XDG_CACHE_HOME/qdc_jit,
// $HOME/.cache/qdc_jit or /tmp/qdc_jit_<uid>: owned by this user, not writable by others), each
// behind a header that names its fingerprint and kernel and hashes its bytes; ensure() loads
// only objects whose header matches.  The missing kernels of a call are compiled in parallel
// child processes (posix_spawn of hipcc; the calling process never execs); one process of a job
// compiles each kernel (a per-kernel flock), the others wait and load it.  Any failure (no
// hipcc, headers changed since the library was built, a compile or load error) turns
// specialization off for the process with one message on stderr: the generic kernel then runs
// every pass, as it does for passes the cap leaves out.
#pragma once

#include <dirent.h>
#include <dlfcn.h>
#include <fcntl.h>
#include <spawn.h>
#include <sys/file.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cerrno>
#include <condition_variable>
#include <csignal>
#include <cstdlib>
#include <deque>
#include <ctime>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "qdc_fusion.hpp"

extern char** environ;

namespace qdc {

// 64-bit FNV-1a of the kernel source: the kernel's name and cache key
inline uint64_t spec_hash(const std::string& s) {
  uint64_t h = 1469598103934665603ull;
  for (unsigned char c : s) h = (h ^ c) * 1099511628211ull;
  return h;
}

// relayouts with immediate LDS offsets (spec_xchg_imm, QDC_SPEC_IMM=1) instead of the XOR form.
// Off by default: the immediate form's reads are bank-conflicted wherever the new layout's low
// lane bits were slots before (its index is a pure bit permutation), and measured slower than
// one v_xor per access on conflict-free swizzled addresses (r3q, C2 n = 28: reverse 2.569 vs
// 2.537 ms, forward 1.278 vs 1.221 ms per launch)
inline bool spec_imm() {
  static const int on = [] {
    const char* e = getenv("QDC_SPEC_IMM");
    return e ? atoi(e) : 0;
  }();
  return on != 0;
}
// Source of one pass program: steps as emitted into the program (relayouts with the layouts
// before and after, stages with their fop), in order.
struct SpecStep {
  bool relayout;
  RqLayout Lc, Ln;  // relayout: current and new layout
  fop F;            // stage: kind (+ FOP_GAMMA), slot case in t1
};
// The generic kernel a specialized one replaces, as the generated source names it.
struct SpecKind {
  bool two;            // two-state (Gamma stages) or one-state
  uint32_t tb, ns;     // thread bits and register slots of a tile (registers per state 2^ns)
  bool bar;            // several waves per tile: block barriers around relayouts
  const char* prefix;  // kernel name prefix (the bench's kernel classes key on it)
  const char* pass;    // the generic kernel's body with the program
  uint32_t threads;
  const char* waves;   // amdgpu_waves_per_eu of the generic kernel
  bool half = false;   // relayouts through half the buffer (spec_xchg_half)
};
#ifndef QDC_F64
// k_rw<true, 2, false, 1, true>: f32 two-state, one wave, five slots
inline SpecKind spec_kind_two(bool half = false) {
  if (half)  // every relayout in two rounds through half the buffer
    return {true, 6, 5, false, "qdc_spec_", "qdc::rw_pass<true, 2, false, 1, true, Prog, true>", 64,
            "QDC_RW_WAVES, QDC_RW_WAVES", true};
  return {true, 6, 5, false, "qdc_spec_", "qdc::rw_pass<true, 2, false, 1, true, Prog>", 64,
          "QDC_RW_WAVES, QDC_RW_WAVES"};
}
// k_rq<false, 256, true>: f32 one-state 2^12 tiles, four waves, prefetching; k_rw<false, 2,
// false, 1, true>: 2^11 tiles (QDC_TILE1_CHUNKS=1024, QDC_RW bit 1), one wave, five slots
// (pf: the next tile prefetched into pinned VGPRs, k_rw<false, 2, true, 1, true>, QDC_RW bit 3)
inline SpecKind spec_kind_one(uint32_t T, bool pf = false, bool half = false) {
  // every relayout in two rounds through half the buffer (8 KiB of LDS per wave): compiled for
  // QDC_RW_WAVES_HALF_ONE [5] waves per SIMD, which LDS now allows (~96 VGPRs, a few spilled;
  // 4 waves at 106 VGPRs measured 0.7-1.0 % slower per step, profiles/r4s)
  if (T == 11 && half && !pf)
    return {false, 6, 5, false, "qdc_specf_", "qdc::rw_pass<false, 2, false, 1, true, Prog, true>", 64,
            "QDC_RW_WAVES_HALF_ONE, QDC_RW_WAVES_HALF_ONE", true};
  if (T == 11 && pf)
    return {false, 6, 5, false, "qdc_specf_", "qdc::rw_pass<false, 2, true, 1, true, Prog>", 64,
            "QDC_RW_WAVES, QDC_RW_WAVES"};
  if (T == 11)
    return {false, 6, 5, false, "qdc_specf_", "qdc::rw_pass<false, 2, false, 1, true, Prog>", 64,
            "QDC_RW_WAVES_ONE, QDC_RW_WAVES_ONE"};
  return {false, 8, 4, true, "qdc_specf_", "qdc::rq_pass<false, 256, true, Prog>", 256,
          "QDC_RQ_PF_WAVES"};
}
#else
// k_rw<true, 1, false, 1>: f64 two-state, one wave
inline SpecKind spec_kind_two(bool = false) {
  return {true, 6, 4, false, "qdc_spec_d_", "qdc::rw_pass<true, 1, false, 1, false, Prog>", 64,
          "QDC_RW_WAVES, QDC_RW_WAVES"};
}
// k_rw<false, 1, false, W>: f64 one-state, W = 1 (2^10 tiles) or 2 (2^11)
inline SpecKind spec_kind_one(uint32_t T, bool = false, bool = false) {
  if (T == 10)
    return {false, 6, 4, false, "qdc_specf_d_", "qdc::rw_pass<false, 1, false, 1, false, Prog>", 64,
            "QDC_RW_WAVES_ONE, QDC_RW_WAVES_ONE"};
  return {false, 7, 4, true, "qdc_specf_d_", "qdc::rw_pass<false, 1, false, 2, false, Prog>", 128,
          "QDC_RW_WAVES_ONE, QDC_RW_WAVES_ONE"};
}
#endif
// The register slot a relayout keeps (the same tile bit in the same slot of both layouts), or
// -1: a half-buffer relayout splits on it (spec_xchg_half).
inline int spec_kept_slot(const RqLayout& Lc, const RqLayout& Ln) {
  if (Lc.ns != Ln.ns) return -1;
  for (uint32_t s = 0; s < Lc.ns; ++s)
    if (Lc.slot[s] == Ln.slot[s] && Lc.slot[s] != ~0u) return (int)s;
  return -1;
}
// A one-state one-wave program whose every relayout keeps a slot runs on half buffers.
inline bool spec_half_ok(const std::vector<SpecStep>& steps) {
  bool any = false;
  for (const SpecStep& s : steps)
    if (s.relayout) {
      any = true;
      if (spec_kept_slot(s.Lc, s.Ln) < 0) return false;
    }
  return any;
}
// the layout's LDS descriptor on the index without tile bit b (rq_descriptor, compressed)
inline rq_layout rq_descriptor_without(const RqLayout& L, uint32_t T, uint32_t b) {
  auto cut = [&](uint32_t i) { return (i & ((1u << b) - 1u)) | ((i >> (b + 1)) << b); };
  rq_layout d{};
  for (uint32_t j = 0; j < (1u << L.ns); ++j) {
    uint32_t idx = 0;
    for (uint32_t s = 0; s < L.ns; ++s)
      if ((j >> s) & 1u) idx |= 1u << L.slot[s];
    d.rp[j] = rq_swz(cut(idx));
  }
  uint32_t th[8];
  const uint32_t nt = L.threads(T, th);
  for (uint32_t k = 0; k < nt; ++k) d.tv[k] = rq_swz(cut(1u << th[k]));
  return d;
}
inline std::string spec_program_source(const std::vector<SpecStep>& steps, uint32_t T, const SpecKind& K) {
  std::string b;
  char tmp[512];
  uint32_t ri = 0;
  const uint32_t TB = K.tb, NR = 1u << K.ns;
  snprintf(tmp, sizeof tmp, "<%u, %s>", TB, K.bar ? "true" : "false");
  const std::string xt = tmp;
  auto arr = [&](const uint32_t* v, uint32_t n) {
    std::string s = "{";
    for (uint32_t i = 0; i < n; ++i) {
      snprintf(tmp, sizeof tmp, "%s%uu", i ? "," : "", v[i]);
      s += tmp;
    }
    return s + "}";
  };
  const std::string nr = std::to_string(NR);
  for (size_t j = 0; j < steps.size(); ++j) {
    const SpecStep& s = steps[j];
    // timing-only ablation builds (QDC_RQ_ABL, qdc_kernels.hpp) drop what the interpreted
    // kernels drop: 1 the stage math, 2 the relayouts, 4 the Gamma accumulation
    if ((QDC_RQ_ABL & 2) && s.relayout) continue;
    if ((QDC_RQ_ABL & 1) && !s.relayout) {
      if (K.two && (s.F.kind & FOP_GAMMA)) ++ri;
      continue;
    }
    if (s.relayout && spec_imm()) {
      // LDS index = bit permutation a(): the current layout's thread bits -> 0..TB-1, slots
      // -> TB..
      uint32_t a[32] = {}, thc[8], thn[8];
      const uint32_t nlc = s.Lc.threads(T, thc);
      s.Ln.threads(T, thn);
      for (uint32_t k = 0; k < TB && k < nlc; ++k) a[thc[k]] = k;
      for (uint32_t q = 0; q < s.Lc.ns; ++q) a[s.Lc.slot[q]] = TB + q;
      uint32_t pn[8], offr[32];
      for (uint32_t k = 0; k < TB; ++k) pn[k] = (uint32_t)sizeof(cx) << a[thn[k]];
      for (uint32_t j = 0; j < NR; ++j) {
        uint32_t o = 0;
        for (uint32_t q = 0; q < s.Ln.ns; ++q)
          if ((j >> q) & 1u) o |= 1u << a[s.Ln.slot[q]];
        offr[j] = o * (uint32_t)sizeof(cx);
      }
      b += "    { constexpr uint32_t pn[" + std::to_string(TB) + "] = " + arr(pn, TB) + ", offr[" + nr +
           "] = " + arr(offr, NR) + ";\n      ";
      b += K.two ? "spec_xchg_imm" + xt + "(xf, E, pn, offr); spec_xchg_imm" + xt + "(xb, E, pn, offr); }\n"
                 : "spec_xchg_imm" + xt + "(x, E, pn, offr); }\n";
      continue;
    }
    if (s.relayout && K.half) {
      const int ks = spec_kept_slot(s.Lc, s.Ln);
      const uint32_t bit = s.Lc.slot[ks];
      const rq_layout c = rq_descriptor_without(s.Lc, T, bit), n = rq_descriptor_without(s.Ln, T, bit);
      b += "    { constexpr uint32_t rc[" + nr + "] = " + arr(c.rp, NR) + ", tc[8] = " + arr(c.tv, 8) +
           ", rn[" + nr + "] = " + arr(n.rp, NR) + ", tn[8] = " + arr(n.tv, 8) + ";\n      ";
      const std::string xh = "spec_xchg_half<" + std::to_string(TB) + ", " + nr + ", " + std::to_string(ks) + ">";
      b += K.two ? xh + "(xf, E, rc, tc, rn, tn); " + xh + "(xb, E, rc, tc, rn, tn); }\n"
                 : xh + "(x, E, rc, tc, rn, tn); }\n";
      continue;
    }
    if (s.relayout) {
      const rq_layout c = rq_descriptor(s.Lc, T), n = rq_descriptor(s.Ln, T);
      b += "    { constexpr uint32_t rc[" + nr + "] = " + arr(c.rp, NR) + ", tc[8] = " + arr(c.tv, 8) +
           ", rn[" + nr + "] = " + arr(n.rp, NR) + ", tn[8] = " + arr(n.tv, 8) + ";\n      ";
      b += K.two ? "spec_xchg" + xt + "(xf, E, rc, tc, rn, tn); spec_xchg" + xt + "(xb, E, rc, tc, rn, tn); }\n"
                 : "spec_xchg" + xt + "(x, E, rc, tc, rn, tn); }\n";
      continue;
    }
    const uint32_t kind = s.F.kind & 7u;
    const bool gamma = K.two && (s.F.kind & FOP_GAMMA) != 0 && !(QDC_RQ_ABL & 4);
    const uint32_t c = s.F.t1;
    std::string tpl = kind == FK_Q1 ? "rq_q1<" + std::to_string(c)
                                    : std::string(kind == FK_DIAG ? "rq_diag<" : "rq_q2<") +
                                          std::to_string(c >> 3) + ", " + std::to_string(c & 7u);
    if (K.two)
      snprintf(tmp, sizeof tmp, "    %s, true, %u>(xf, xb, E.mats + E.ops[%zu].mat, %s, &E.accw[%u][0]);\n",
               tpl.c_str(), NR, j, gamma ? "true" : "false", ri);
    else
      snprintf(tmp, sizeof tmp, "    %s, false, %u>(x, x, E.mats + E.ops[%zu].mat, false, nullptr);\n",
               tpl.c_str(), NR, j);
    b += tmp;
    if (gamma) ++ri;
  }
  return b;
}
inline std::string spec_kernel_source(const std::string& name, const std::string& body, const SpecKind& K) {
  const std::string R = std::to_string(1u << K.ns);
  const std::string args =
      K.two ? "qdc::cx (&xf)[" + R + "], qdc::cx (&xb)[" + R + "], const qdc::SpecEnv& E"
            : "qdc::cx (&x)[" + R + "], const qdc::SpecEnv& E";
  return "#define QDC_SPEC_TU 1\n#include \"qdc_spec.hpp\"\n"
         "namespace {\n"
         "struct Prog {\n"
         "  __device__ __forceinline__ void operator()(" + args + ") const {\n"
         "    using namespace qdc;\n" +
         body +
         "  }\n"
         "};\n"
         "}  // namespace\n"
         "extern \"C\" __global__ __launch_bounds__(" + std::to_string(K.threads) +
         ") __attribute__((amdgpu_waves_per_eu(" + K.waves + ")))\n"
         "void " + name + "(qdc::chunk* __restrict__ f, qdc::chunk* __restrict__ b,\n"
         "    const qdc::fop* __restrict__ ops, const qdc::cx* __restrict__ mats, qdc::fgeo fg,\n"
         "    uint32_t l0, qdc::cx* __restrict__ partials, uint64_t slot_stride) {\n"
         "  " + K.pass + "(f, b, ops, mats, fg, l0, partials, slot_stride);\n"
         "}\n";
}

// one generated kernel: name, source, and its function per device once loaded
struct SpecEntry {
  std::string name, src;
  std::map<int, hipFunction_t> fn;
  uint64_t epoch = 0;  // last call (spec_load) that counted it
};

// FNV-1a continued over more bytes
inline uint64_t fnv_more(uint64_t h, const void* p, size_t n) {
  const unsigned char* c = static_cast<const unsigned char*>(p);
  for (size_t i = 0; i < n; ++i) h = (h ^ c[i]) * 1099511628211ull;
  return h;
}
inline bool read_file(const std::string& path, std::string& out) {
  FILE* fp = fopen(path.c_str(), "rb");
  if (!fp) return false;
  out.clear();
  char b[65536];
  size_t k;
  while ((k = fread(b, 1, sizeof b, fp)) > 0) out.append(b, k);
  const bool ok = !ferror(fp);
  fclose(fp);
  return ok;
}

// The kernel headers a generated source compiles against: every csrc/*.hpp and include/qdc/*.h,
// hashed as (relative path, NUL, bytes, NUL) in sorted path order.  csrc/src_fp.py computes the
// same at build time (QDC_SRC_FP), so a library can tell that the headers next to it are no
// longer the ones it was built from.
inline bool spec_source_fp(const std::string& csrc, const std::string& inc, uint64_t& out) {
  std::vector<std::pair<std::string, std::string>> files;  // (relative name, path)
  auto scan = [&](const std::string& dir, const std::string& rel, const char* ext) {
    DIR* d = opendir(dir.c_str());
    if (!d) return false;
    const size_t el = strlen(ext);
    while (dirent* e = readdir(d)) {
      const std::string nm = e->d_name;
      if (nm.size() > el && nm.compare(nm.size() - el, el, ext) == 0 && nm[0] != '.')
        files.emplace_back(rel + nm, dir + "/" + nm);
    }
    closedir(d);
    return true;
  };
  if (!scan(csrc, "csrc/", ".hpp") || !scan(inc + "/qdc", "include/qdc/", ".h")) return false;
  std::sort(files.begin(), files.end());
  uint64_t h = 1469598103934665603ull;
  std::string body;
  for (const auto& f : files) {
    if (!read_file(f.second, body)) return false;
    h = fnv_more(h, f.first.c_str(), f.first.size() + 1);
    h = fnv_more(h, body.data(), body.size());
    h = fnv_more(h, "", 1);
  }
  out = h;
  return true;
}

// the library's own compile-time switches, so the kernels agree with it
#ifndef QDC_NT_LOAD
#define QDC_NT_LOAD 1
#endif
#ifndef QDC_NT_STORE
#define QDC_NT_STORE 1
#endif
#ifndef QDC_RW_WAVES_HALF_ONE
#define QDC_RW_WAVES_HALF_ONE 5
#endif
#ifndef QDC_PK_ASM  // (qdc_kernels.hpp; f64 builds never read them)
#define QDC_PK_ASM 1
#endif
#ifndef QDC_PK_VASM
#define QDC_PK_VASM 1
#endif
inline std::string spec_defines() {
  char b[512];
  snprintf(b, sizeof b,
           "-DQDC_DYN_TAIL=%d -DQDC_FMAX_OPS=%d -DQDC_FMAX_GRAD_RQ=%d -DQDC_RQ_PF_WAVES=%d "
           "-DQDC_RW_WAVES=%d -DQDC_RW_WAVES_ONE=%d -DQDC_RQ_ABL=%d -DQDC_RQ_GSPLIT=%d "
           "-DQDC_NT_LOAD=%d -DQDC_NT_STORE=%d -DQDC_RW_WAVES_HALF_ONE=%d -DQDC_PK_ASM=%d -DQDC_PK_VASM=%d "
           "-DQDC_MATVEC_N=%d%s",
           (int)QDC_DYN_TAIL, (int)FMAX_OPS, (int)FMAX_GRAD_RQ, (int)QDC_RQ_PF_WAVES,
           (int)QDC_RW_WAVES, (int)QDC_RW_WAVES_ONE, (int)QDC_RQ_ABL, (int)QDC_RQ_GSPLIT,
           (int)QDC_NT_LOAD, (int)QDC_NT_STORE, (int)QDC_RW_WAVES_HALF_ONE, (int)QDC_PK_ASM, (int)QDC_PK_VASM, (int)QDC_MATVEC_N,
           sizeof(real) == 8 ? " -DQDC_F64" : "");
  return b;
}
// hipcc options of every specialized kernel besides the defines and include paths
inline const char* spec_cflags() { return "--genco -O3 -std=c++17 --offload-arch=gfx950"; }
// The build fingerprint that goes into every kernel name: the defines, the compiler's identity
// (its path and --version text), the options and the header bytes.  Two libraries that differ
// in any of them never share a code object in one cache directory.
inline uint64_t spec_fingerprint(const std::string& defines, const std::string& compiler,
                                 uint64_t source_fp) {
  uint64_t h = 1469598103934665603ull;
  const std::string s = defines + "\n" + compiler + "\n" + spec_cflags() + "\n";
  h = fnv_more(h, s.data(), s.size());
  return fnv_more(h, &source_fp, sizeof source_fp);
}
// kernel name: prefix + hash of the build fingerprint, the generic kernel and the program
inline std::string spec_kernel_name_fp(const std::string& body, const SpecKind& K, uint64_t fp) {
  char nm[48];
  uint64_t h = spec_hash(std::string(K.pass) + "\n" + body);
  h = fnv_more(h, &fp, sizeof fp);
  snprintf(nm, sizeof nm, "%s%016llx", K.prefix, (unsigned long long)h);
  return nm;
}

#ifndef QDC_SRC_FP
#define QDC_SRC_FP 0ull  // not built by csrc/Makefile: the header check is skipped
#endif

// A code object on disk: this header, then hipcc's output.  ensure() loads an object only when
// the header names the current build fingerprint and the kernel, and the bytes are whole.
struct JitObjHeader {
  char magic[8];
  uint64_t fp, name_hash, size, body_hash;
};
static_assert(sizeof(JitObjHeader) == 40, "code-object header layout");
constexpr char JIT_MAGIC[8] = {'Q', 'D', 'C', 'J', 'I', 'T', '2', '\0'};

// counters of this process's specialized-kernel cache (qdc_jit_stats)
struct JitStats {
  uint64_t queued = 0;    // kernels waiting for (or in) the background compiler
  uint64_t compiled = 0;  // kernels this process compiled
  uint64_t waited = 0;    // kernels another process was compiling when this one needed them
  uint64_t loaded = 0;    // (kernel, device) loads
  double compile_s = 0, wait_s = 0, ensure_s = 0;
};

// hipcc children of the background compiler, killed at process exit (an exit during a long
// background compile leaves no orphaned compiles behind)
inline std::atomic<pid_t>* jit_children() {
  static std::atomic<pid_t> pids[16];
  return pids;
}
inline void jit_kill_children() {
  for (int k = 0; k < 16; ++k) {
    const pid_t p = jit_children()[k].exchange(0);
    if (p > 0) kill(p, SIGKILL);
  }
}

class SpecJit {
 public:
  static SpecJit& get() {
    // never destroyed: the background compiler's thread may still run at static destruction
    static SpecJit* j = new SpecJit;
    return *j;
  }
  // Asynchronous form of ensure() for programs with more distinct kernels than a call should
  // wait for (deep random circuits, Circuit::spec_load): the kernels whose objects exist (this
  // process, the cache or the prebuilt directory) are loaded on `device` now; the missing ones
  // are queued for a background thread that compiles them (the same per-kernel locks and cache),
  // and their passes run the generic kernel until a later call finds the object.  f32
  // specialized and generic passes are bit-identical, so results do not depend on the timing.
  void ensure_async(int device, const std::vector<std::string>& names,
                    const std::vector<std::string>& srcs, std::vector<hipFunction_t>& fns) {
    std::lock_guard<std::mutex> lk(mu);
    const double t0 = now();
    fns.assign(names.size(), nullptr);
    if (!init()) return;
    for (size_t i = 0; i < names.size(); ++i) {
      auto it = loaded.find({device, names[i]});
      if (it != loaded.end()) {
        fns[i] = it->second;
        continue;
      }
      if (!image(names[i])) {
        if (!pending.count(names[i])) {
          pending.insert(names[i]);
          queue.push_back({names[i], srcs[i]});
        }
        continue;
      }
      hipModule_t mod = nullptr;
      hipFunction_t fn = nullptr;
      if (hipModuleLoadData(&mod, image(names[i])->data()) != hipSuccess ||
          hipModuleGetFunction(&fn, mod, names[i].c_str()) != hipSuccess) {
        (void)hipGetLastError();
        disable("cannot load " + obj_path(names[i]));
        fns.assign(names.size(), nullptr);
        break;
      }
      ++stats.loaded;
      fns[i] = loaded.emplace(std::make_pair(device, names[i]), fn).first->second;
    }
    stats.queued = pending.size();
    if (!queue.empty() && !worker_on && state > 0) {
      worker_on = true;
      static bool hooked = (std::atexit(jit_kill_children), true);
      (void)hooked;
      std::thread([this] { background(); }).detach();
    }
    stats.ensure_s += now() - t0;
  }
  // Wait until the background compiler has drained its queue or `timeout_s` passed; returns the
  // kernels still queued.
  size_t wait_async(double timeout_s) {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait_for(lk, std::chrono::duration<double>(timeout_s < 0 ? 0 : timeout_s),
                [this] { return !worker_on; });
    return pending.size();
  }
  // the build fingerprint (0 while specialization is off)
  uint64_t fingerprint() {
    std::lock_guard<std::mutex> lk(mu);
    return init() ? fp : 0;
  }
  // Kernels of the given names / sources on `device` (the current device), compiling and
  // loading the missing ones; fns[i] = nullptr where specialization is off.
  void ensure(int device, const std::vector<std::string>& names,
              const std::vector<std::string>& srcs, std::vector<hipFunction_t>& fns) {
    std::lock_guard<std::mutex> lk(mu);
    const double t0 = now();
    fns.assign(names.size(), nullptr);
    if (!init()) return;
    std::vector<size_t> todo;
    for (size_t i = 0; i < names.size(); ++i) {
      auto it = loaded.find({device, names[i]});
      if (it != loaded.end()) {
        fns[i] = it->second;
        continue;
      }
      bool dup = false;
      for (size_t k : todo) dup = dup || names[k] == names[i];
      if (!dup && !image(names[i])) todo.push_back(i);
    }
    if (!todo.empty() && !obtain(names, srcs, todo)) {
      stats.ensure_s += now() - t0;
      return;
    }
    for (size_t i = 0; i < names.size(); ++i) {
      if (fns[i]) continue;
      auto it = loaded.find({device, names[i]});
      if (it == loaded.end()) {
        hipModule_t mod = nullptr;
        hipFunction_t fn = nullptr;
        const std::vector<char>* img = image(names[i]);
        if (!img || hipModuleLoadData(&mod, img->data()) != hipSuccess ||
            hipModuleGetFunction(&fn, mod, names[i].c_str()) != hipSuccess) {
          (void)hipGetLastError();
          disable("cannot load " + obj_path(names[i]));
          fns.assign(names.size(), nullptr);
          stats.ensure_s += now() - t0;
          return;
        }
        ++stats.loaded;
        it = loaded.emplace(std::make_pair(device, names[i]), fn).first;
      }
      fns[i] = it->second;
    }
    stats.ensure_s += now() - t0;
  }
  bool enabled() {
    std::lock_guard<std::mutex> lk(mu);
    return init();
  }
  // compile without loading (host-only test hook): nullptr when every code object is valid after
  const char* compile_only(const std::vector<std::string>& names,
                           const std::vector<std::string>& srcs) {
    std::lock_guard<std::mutex> lk(mu);
    if (!init()) return "specialization unavailable (no hipcc, kernel sources or cache directory)";
    std::vector<size_t> todo;
    for (size_t i = 0; i < names.size(); ++i)
      if (!image(names[i])) todo.push_back(i);
    if (!todo.empty() && !obtain(names, srcs, todo)) return "hipcc failed";
    return nullptr;
  }
  std::string code_object(const std::string& name) const { return obj_path(name); }
  std::string cache_dir() {
    std::lock_guard<std::mutex> lk(mu);
    return init() ? dir : std::string();
  }
  JitStats counters() {
    std::lock_guard<std::mutex> lk(mu);
    return stats;
  }
  // processes of this job on the node (ranks): the default compile parallelism is shared
  void set_processes(int p) {
    std::lock_guard<std::mutex> lk(mu);
    procs = std::max(procs, p);
  }

 private:
  std::mutex mu;
  std::condition_variable cv;
  // the background compiler (ensure_async): queued kernels (name, source), their names, whether
  // its thread runs
  std::deque<std::pair<std::string, std::string>> queue;
  std::set<std::string> pending;
  bool worker_on = false;
  // Background compiles, one batch of the compile parallelism at a time under the lock (ensure()
  // and the runtime wait at most one batch: seconds); kernels another process of the job is
  // compiling are not waited for under the lock (their flock waits can last minutes) but queued
  // again behind the rest, and a batch of nothing but those sleeps without the lock; exits when
  // the queue is empty or specialization was switched off.
  void background() {
    for (;;) {
      bool idle = false;
      {
        std::lock_guard<std::mutex> lk(mu);
        if (queue.empty() || state <= 0) {
          queue.clear();
          pending.clear();
          stats.queued = 0;
          worker_on = false;
          cv.notify_all();
          return;
        }
        std::vector<std::string> names, srcs;
        std::vector<size_t> todo;
        size_t take = (size_t)jobs_now();
        if (const char* e = getenv("QDC_JIT_ASYNC_JOBS")) take = (size_t)std::max(1, atoi(e));
        take = std::min(queue.size(), take);
        for (size_t k = 0; k < take; ++k) {
          names.push_back(queue.front().first);
          srcs.push_back(queue.front().second);
          todo.push_back(k);
          queue.pop_front();
        }
        std::vector<size_t> deferred;
        (void)obtain(names, srcs, todo, &deferred);  // (a failure disables specialization: loop ends)
        std::vector<bool> again(names.size(), false);
        for (size_t k : deferred) {
          again[k] = true;
          queue.push_back({names[k], srcs[k]});
        }
        for (size_t k = 0; k < names.size(); ++k)
          if (!again[k]) pending.erase(names[k]);
        stats.queued = pending.size();
        idle = !deferred.empty() && deferred.size() == names.size();
      }
      cv.notify_all();
      if (idle) usleep(50000);
    }
  }
  std::map<std::pair<int, std::string>, hipFunction_t> loaded;
  std::map<std::string, std::vector<char>> images;  // validated code objects (kept for the process)
  std::string hipcc, csrc, inc, dir;
  // code objects compiled ahead of time (in-tree <pkg>/jit-prebuilt, written by build() through
  // qdc_precompile; QDC_JIT_PREBUILT names another, 0 none): read-only, searched after `dir`,
  // validated like the cache's own objects (fingerprint, kernel name, byte hash); used only when
  // owned by this user and writable by no one else
  std::string prebuilt;
  uint64_t fp = 0;
  int state = 0;  // 0 unknown, 1 on, -1 off
  int procs = 1;
  JitStats stats;
  static double now() {
    timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + 1e-9 * ts.tv_nsec;
  }
  std::string obj_path(const std::string& name) const { return dir + "/" + name + ".qco"; }
  std::string lock_path(const std::string& name) const { return dir + "/" + name + ".lock"; }
  void disable(const std::string& why) {
    if (state != -1) fprintf(stderr, "qdc: specialized passes off (%s)\n", why.c_str());
    state = -1;
  }
  // the validated code object of `name` (cached in memory), or nullptr when the file is
  // missing, from another build, truncated or otherwise not this kernel's
  const std::vector<char>* image(const std::string& name) {
    auto it = images.find(name);
    if (it != images.end()) return &it->second;
    std::string raw;
    // the cache directory, then the read-only prebuilt directory (build(): qdc_precompile)
    if ((!read_file(obj_path(name), raw) || raw.size() <= sizeof(JitObjHeader)) &&
        (prebuilt.empty() || !read_file(prebuilt + "/" + name + ".qco", raw) ||
         raw.size() <= sizeof(JitObjHeader)))
      return nullptr;
    JitObjHeader h;
    memcpy(&h, raw.data(), sizeof h);
    const char* body = raw.data() + sizeof h;
    const size_t n = raw.size() - sizeof h;
    if (memcmp(h.magic, JIT_MAGIC, 8) != 0 || h.fp != fp || h.name_hash != spec_hash(name) ||
        h.size != n || h.body_hash != fnv_more(1469598103934665603ull, body, n))
      return nullptr;
    return &images.emplace(name, std::vector<char>(body, body + n)).first->second;
  }
  // A cache directory no other user can write into: not a symlink, owned by this user, not
  // group/world-writable (a default location: no group/world access at all).
  static bool secure_dir(const std::string& d, bool strict, std::string& why) {
    mkdir(d.c_str(), 0700);
    struct stat st;
    if (lstat(d.c_str(), &st) != 0) {
      why = d + ": cannot be created";
      return false;
    }
    if (S_ISLNK(st.st_mode) || !S_ISDIR(st.st_mode)) {
      why = d + ": not a directory";
      return false;
    }
    if (st.st_uid != geteuid()) {
      why = d + ": owned by another user";
      return false;
    }
    if (st.st_mode & (strict ? 077 : 022)) {
      why = d + (strict ? ": accessible to other users" : ": writable by other users");
      return false;
    }
    if (access(d.c_str(), W_OK | X_OK) != 0) {
      why = d + ": not writable";
      return false;
    }
    return true;
  }
  // QDC_JIT_DIR, else $XDG_CACHE_HOME/qdc_jit, $HOME/.cache/qdc_jit, /tmp/qdc_jit_<uid>: the
  // first that passes secure_dir
  bool choose_dir(std::string& why) {
    if (const char* d = getenv("QDC_JIT_DIR")) {
      dir = d;
      return secure_dir(dir, false, why);
    }
    std::vector<std::string> cand;
    const char* xdg = getenv("XDG_CACHE_HOME");
    if (xdg && xdg[0] == '/') cand.push_back(std::string(xdg) + "/qdc_jit");
    const char* home = getenv("HOME");
    if (home && home[0] == '/') {
      mkdir((std::string(home) + "/.cache").c_str(), 0700);
      cand.push_back(std::string(home) + "/.cache/qdc_jit");
    }
    cand.push_back("/tmp/qdc_jit_" + std::to_string((unsigned)geteuid()));
    std::string w;
    for (const std::string& c : cand) {
      if (secure_dir(c, true, w)) {
        dir = c;
        return true;
      }
      why += (why.empty() ? "" : "; ") + w;
    }
    return false;
  }
  // the standard output + error of a child (posix_spawn: this process never execs)
  static bool run_capture(const std::vector<std::string>& args, std::string& out) {
    int fd[2];
    if (pipe(fd) != 0) return false;
    posix_spawn_file_actions_t fa;
    posix_spawn_file_actions_init(&fa);
    posix_spawn_file_actions_adddup2(&fa, fd[1], 1);
    posix_spawn_file_actions_adddup2(&fa, fd[1], 2);
    posix_spawn_file_actions_addclose(&fa, fd[0]);
    posix_spawn_file_actions_addclose(&fa, fd[1]);
    std::vector<char*> argv;
    for (const std::string& a : args) argv.push_back(const_cast<char*>(a.c_str()));
    argv.push_back(nullptr);
    pid_t pid = 0;
    const int rc = posix_spawn(&pid, args[0].c_str(), &fa, nullptr, argv.data(), environ);
    posix_spawn_file_actions_destroy(&fa);
    close(fd[1]);
    out.clear();
    if (rc == 0) {
      char b[4096];
      ssize_t k;
      while ((k = read(fd[0], b, sizeof b)) > 0 || (k < 0 && errno == EINTR))
        if (k > 0) out.append(b, (size_t)k);
    }
    close(fd[0]);
    int status = 0;
    if (rc != 0 || waitpid(pid, &status, 0) < 0) return false;
    return WIFEXITED(status) && WEXITSTATUS(status) == 0;
  }
  bool init() {
    if (state) return state > 0;
    Dl_info di{};
    if (!dladdr((const void*)&spec_hash, &di) || !di.dli_fname) {
      disable("library path unknown");
      return false;
    }
    std::string lib = di.dli_fname;  // <pkg>/lib/libqdc_f32.so
    const size_t cut = lib.rfind('/');
    const std::string libdir = cut == std::string::npos ? "." : lib.substr(0, cut);
    csrc = libdir + "/../csrc";
    inc = libdir + "/../../include";
    if (const char* sd = getenv("QDC_SRC_DIR")) {  // a library built elsewhere (A/B builds)
      csrc = sd;
      inc = std::string(sd) + "/../../include";
    }
    const char* h = getenv("QDC_HIPCC");
    const char* rp = getenv("ROCM_PATH");
    hipcc = h ? h : (rp ? std::string(rp) + "/bin/hipcc" : "/opt/rocm/bin/hipcc");
    if (!exists(csrc + "/qdc_spec.hpp") || access(hipcc.c_str(), X_OK) != 0) {
      disable("no hipcc or kernel sources next to the library");
      return false;
    }
    uint64_t sfp = 0;
    if (!spec_source_fp(csrc, inc, sfp)) {
      disable("cannot read the kernel headers in " + csrc);
      return false;
    }
    if ((uint64_t)QDC_SRC_FP != 0 && sfp != (uint64_t)QDC_SRC_FP) {
      disable("the kernel headers in " + csrc + " are not the ones this library was built from");
      return false;
    }
    std::string ver;
    if (!run_capture({hipcc, "--version"}, ver)) {
      disable(hipcc + " --version failed");
      return false;
    }
    std::string why;
    if (!choose_dir(why)) {
      disable("no private cache directory (" + why + ")");
      return false;
    }
    // the compiler's identity as the fingerprint sees it: its canonical path and the version
    // lines of its --version text, so a run under a profiler (another ROCM_PATH spelling, a
    // preloaded tool writing to the child's stdout) names the same kernels as a plain run
    std::string ident;
    {
      char rbuf[4096];
      ident = realpath(hipcc.c_str(), rbuf) ? std::string(rbuf) : hipcc;
      size_t p0 = 0;
      while (p0 < ver.size()) {
        size_t p1 = ver.find('\n', p0);
        if (p1 == std::string::npos) p1 = ver.size();
        const std::string line = ver.substr(p0, p1 - p0);
        for (const char* key : {"HIP version", "AMD clang version", "clang version", "Target:"})
          if (line.rfind(key, 0) == 0) {
            ident += "\n" + line;
            break;
          }
        p0 = p1 + 1;
      }
    }
    fp = spec_fingerprint(spec_defines(), ident, sfp);
    {
      const char* pe = getenv("QDC_JIT_PREBUILT");
      std::string p = pe ? std::string(pe) : libdir + "/../jit-prebuilt";
      struct stat st;
      if ((pe && std::string(pe) == "0") || p == dir || lstat(p.c_str(), &st) != 0 ||
          !S_ISDIR(st.st_mode) || st.st_uid != geteuid() || (st.st_mode & 022))
        p.clear();
      prebuilt = p;
    }
    state = 1;
    return true;
  }
  static bool exists(const std::string& p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0;
  }
  // compile parallelism of this process: the node's hipcc processes shared by the job's ranks
  int jobs_now() const {
    int jobs = std::min((int)std::thread::hardware_concurrency(), 16) / procs;
    if (const char* e = getenv("QDC_JIT_JOBS")) jobs = atoi(e);
    return std::max(1, std::min(jobs, 16));
  }
  // The missing kernels `todo`: one process compiles each.  Work-stealing over per-kernel locks
  // (flock, released by the kernel if the holder dies): take up to this process's compile
  // parallelism of the free locks whose object is still missing, compile them, release, repeat;
  // when every remaining kernel is held by another process, wait for one, then load it — or
  // compile it here if that process failed.  So the ranks of a job share the compiles instead of
  // the first one taking them all.
  // deferred (background compiler): kernels left only because other processes hold their
  // locks are returned there instead of waited for
  bool obtain(const std::vector<std::string>& names, const std::vector<std::string>& srcs,
              const std::vector<size_t>& todo, std::vector<size_t>* deferred = nullptr) {
    auto lock_fd = [&](size_t i) {
      return open(lock_path(names[i]).c_str(), O_RDWR | O_CREAT | O_CLOEXEC | O_NOFOLLOW, 0600);
    };
    auto release = [](int fd) {
      flock(fd, LOCK_UN);
      close(fd);
    };
    double wait_lim = 900;
    if (const char* e = getenv("QDC_JIT_WAIT_S")) wait_lim = atof(e);
    const int jobs = jobs_now();
    std::vector<size_t> rem = todo;
    // start at a process-dependent kernel: concurrent ranks begin on different locks
    if (!rem.empty()) std::rotate(rem.begin(), rem.begin() + (size_t)getpid() % rem.size(), rem.end());
    while (!rem.empty()) {
      std::vector<size_t> batch, left;
      std::vector<int> held;
      for (size_t i : rem) {
        if (image(names[i])) continue;  // done (here or elsewhere)
        if ((int)batch.size() >= jobs) {
          left.push_back(i);
          continue;
        }
        const int fd = lock_fd(i);
        if (fd < 0) {
          for (int h : held) release(h);
          disable("cannot create " + lock_path(names[i]));
          return false;
        }
        if (flock(fd, LOCK_EX | LOCK_NB) != 0) {  // another process compiles it
          close(fd);
          left.push_back(i);
          continue;
        }
        if (image(names[i])) {  // finished between the check and the lock
          release(fd);
          continue;
        }
        batch.push_back(i);
        held.push_back(fd);
      }
      if (!batch.empty()) {
        const bool ok = compile(names, srcs, batch);
        for (int h : held) release(h);
        if (!ok) return false;
        rem = left;
        continue;
      }
      if (left.empty()) break;
      if (deferred) {
        *deferred = left;
        return true;
      }
      // every remaining kernel is being compiled elsewhere: wait for the first of them
      const size_t i = left.front();
      const int fd = lock_fd(i);
      if (fd < 0) {
        disable("cannot create " + lock_path(names[i]));
        return false;
      }
      const double t0 = now();
      ++stats.waited;
      while (flock(fd, LOCK_EX | LOCK_NB) != 0) {
        if (now() - t0 > wait_lim) {
          close(fd);
          stats.wait_s += now() - t0;
          disable("timed out waiting for another process compiling " + names[i]);
          return false;
        }
        usleep(20000);
      }
      stats.wait_s += now() - t0;
      const bool ok = image(names[i]) || compile(names, srcs, {i});
      release(fd);
      if (!ok) return false;
      rem = left;
    }
    return true;
  }
  // write `elf` as the code object of `name` (header + bytes) by atomic rename
  bool publish(const std::string& name, const std::string& elf, const std::string& tag) {
    JitObjHeader h;
    memcpy(h.magic, JIT_MAGIC, 8);
    h.fp = fp;
    h.name_hash = spec_hash(name);
    h.size = elf.size();
    h.body_hash = fnv_more(1469598103934665603ull, elf.data(), elf.size());
    const std::string tmp = obj_path(name) + "." + tag + ".tmp";
    FILE* fo = fopen(tmp.c_str(), "wb");
    if (!fo) return false;
    bool ok = fwrite(&h, sizeof h, 1, fo) == 1 && fwrite(elf.data(), 1, elf.size(), fo) == elf.size();
    ok = (fclose(fo) == 0) && ok;
    if (!ok || rename(tmp.c_str(), obj_path(name).c_str()) != 0) {
      unlink(tmp.c_str());
      return false;
    }
    return true;
  }
  bool compile(const std::vector<std::string>& names, const std::vector<std::string>& srcs,
               const std::vector<size_t>& todo) {
    const double t0 = now();
    const int jobs = jobs_now();
    const char* keep_env = getenv("QDC_JIT_KEEP");  // keep sources and logs of good compiles
    const bool keep = keep_env && atoi(keep_env) != 0;
    struct Job {
      pid_t pid;
      size_t i;
      std::string src, out;
    };
    std::vector<Job> run;
    size_t next = 0;
    bool ok = true;
    const std::string tag = std::to_string((long)getpid());
    const std::string defs = spec_defines(), flags = spec_cflags();
    auto reap = [&]() {
      int status = 0;
      const pid_t p = waitpid(run.front().pid, &status, 0);
      for (int k = 0; k < 16; ++k) {
        pid_t z = run.front().pid;
        if (jit_children()[k].compare_exchange_strong(z, 0)) break;
      }
      Job j = run.front();
      run.erase(run.begin());
      std::string elf;
      const bool good = p >= 0 && WIFEXITED(status) && WEXITSTATUS(status) == 0 &&
                        read_file(j.out, elf) && !elf.empty() && publish(names[j.i], elf, tag);
      unlink(j.out.c_str());
      if (!good) {
        ok = false;  // the source and the log stay for inspection
        return;
      }
      ++stats.compiled;
      if (!keep) {
        unlink(j.src.c_str());
        unlink((j.src + ".log").c_str());
      }
    };
    while (next < todo.size() || !run.empty()) {
      if (ok && next < todo.size() && (int)run.size() < jobs) {
        const size_t i = todo[next++];
        Job j{0, i, dir + "/" + names[i] + "." + tag + ".hip", dir + "/" + names[i] + "." + tag + ".elf"};
        FILE* fp_src = fopen(j.src.c_str(), "w");
        if (!fp_src) {
          ok = false;
          continue;
        }
        fputs(srcs[i].c_str(), fp_src);
        fclose(fp_src);
        std::vector<std::string> args = {hipcc};
        for (const std::string* s : {&flags, &defs}) {
          size_t p = 0;
          while (p < s->size()) {
            size_t q = s->find(' ', p);
            if (q == std::string::npos) q = s->size();
            if (q > p) args.push_back(s->substr(p, q - p));
            p = q + 1;
          }
        }
        for (const std::string& a : {"-I" + inc, "-I" + csrc, std::string("-o"), j.out, j.src}) args.push_back(a);
        std::vector<char*> argv;
        for (auto& a : args) argv.push_back(const_cast<char*>(a.c_str()));
        argv.push_back(nullptr);
        posix_spawn_file_actions_t fa;
        posix_spawn_file_actions_init(&fa);
        const std::string log = j.src + ".log";
        posix_spawn_file_actions_addopen(&fa, 1, log.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0600);
        posix_spawn_file_actions_adddup2(&fa, 1, 2);
        const int rc = posix_spawn(&j.pid, hipcc.c_str(), &fa, nullptr, argv.data(), environ);
        posix_spawn_file_actions_destroy(&fa);
        if (rc != 0) {
          ok = false;
          continue;
        }
        for (int k = 0; k < 16; ++k) {  // (killed at exit if still running)
          pid_t z = 0;
          if (jit_children()[k].compare_exchange_strong(z, j.pid)) break;
        }
        run.push_back(j);
        continue;
      }
      if (!run.empty()) reap();
      else break;
    }
    stats.compile_s += now() - t0;
    if (!ok) disable("hipcc failed on a pass kernel (sources and logs in " + dir + ")");
    return ok;
  }
};

// kernel name of a program under this library's build fingerprint
inline std::string spec_kernel_name(const std::string& body, const SpecKind& K) {
  return spec_kernel_name_fp(body, K, SpecJit::get().fingerprint());
}

}  // namespace qdc
