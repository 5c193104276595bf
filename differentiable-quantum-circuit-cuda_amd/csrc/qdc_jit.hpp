// qdc_jit.hpp — the specialized pass kernels (qdc_spec.hpp; two-state reverse passes and
// one-state forward passes): source per pass program, compiled with hipcc for gfx950 on first
// use, cached on disk and per device.
//
// A pass program becomes a functor of straight-line stage calls; its source text (hashed)
// names the kernel, so passes with the same program share one kernel, across circuits and
// processes (the code objects live in QDC_JIT_DIR, default /tmp/qdc_jit_<uid>).  The missing
// kernels of a call are compiled in parallel child processes (posix_spawn of hipcc; the
// calling process never execs), then loaded with hipModuleLoad.  Any failure (no hipcc, a
// compile error, a load error) turns specialization off for the process with one message on
// stderr: the generic kernel then runs every pass, as it does for passes the cap leaves out.
#pragma once

#include <dlfcn.h>
#include <fcntl.h>
#include <spawn.h>
#include <sys/stat.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
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
};
#ifndef QDC_F64
// k_rw<true, 2, false, 1, true>: f32 two-state, one wave, five slots
inline SpecKind spec_kind_two() {
  return {true, 6, 5, false, "qdc_spec_", "qdc::rw_pass<true, 2, false, 1, true, Prog>", 64,
          "QDC_RW_WAVES, QDC_RW_WAVES"};
}
// k_rq<false, 256, true>: f32 one-state, four waves, prefetching
inline SpecKind spec_kind_one(uint32_t) {
  return {false, 8, 4, true, "qdc_specf_", "qdc::rq_pass<false, 256, true, Prog>", 256,
          "QDC_RQ_PF_WAVES"};
}
#else
// k_rw<true, 1, false, 1>: f64 two-state, one wave
inline SpecKind spec_kind_two() {
  return {true, 6, 4, false, "qdc_spec_d_", "qdc::rw_pass<true, 1, false, 1, false, Prog>", 64,
          "QDC_RW_WAVES, QDC_RW_WAVES"};
}
// k_rw<false, 1, false, W>: f64 one-state, W = 1 (2^10 tiles) or 2 (2^11)
inline SpecKind spec_kind_one(uint32_t T) {
  if (T == 10)
    return {false, 6, 4, false, "qdc_specf_d_", "qdc::rw_pass<false, 1, false, 1, false, Prog>", 64,
            "QDC_RW_WAVES_ONE, QDC_RW_WAVES_ONE"};
  return {false, 7, 4, true, "qdc_specf_d_", "qdc::rw_pass<false, 1, false, 2, false, Prog>", 128,
          "QDC_RW_WAVES_ONE, QDC_RW_WAVES_ONE"};
}
#endif
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
    if (s.relayout) {
      const rq_layout c = rq_descriptor(s.Lc, T), n = rq_descriptor(s.Ln, T);
      b += "    { constexpr uint32_t rc[" + nr + "] = " + arr(c.rp, NR) + ", tc[8] = " + arr(c.tv, 8) +
           ", rn[" + nr + "] = " + arr(n.rp, NR) + ", tn[8] = " + arr(n.tv, 8) + ";\n      ";
      b += K.two ? "spec_xchg" + xt + "(xf, E, rc, tc, rn, tn); spec_xchg" + xt + "(xb, E, rc, tc, rn, tn); }\n"
                 : "spec_xchg" + xt + "(x, E, rc, tc, rn, tn); }\n";
      continue;
    }
    const uint32_t kind = s.F.kind & 7u;
    const bool gamma = K.two && (s.F.kind & FOP_GAMMA) != 0;
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
// kernel name (prefix + hash of the generic kernel and the program) and source
inline std::string spec_kernel_name(const std::string& body, const SpecKind& K) {
  char nm[48];
  snprintf(nm, sizeof nm, "%s%016llx", K.prefix,
           (unsigned long long)spec_hash(std::string(K.pass) + "\n" + body));
  return nm;
}
inline std::string spec_kernel_source(const std::string& name, const std::string& body, const SpecKind& K) {
  const std::string R = std::to_string(1u << K.ns);
  const std::string args =
      K.two ? "qdc::cx (&xf)[" + R + "], qdc::cx (&xb)[" + R + "], const qdc::SpecEnv& E"
            : "qdc::cx (&x)[" + R + "], const qdc::SpecEnv& E";
  return "#include \"qdc_spec.hpp\"\n"
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

class SpecJit {
 public:
  static SpecJit& get() {
    static SpecJit j;
    return j;
  }
  // Kernels of the given names / sources on `device` (the current device), compiling and
  // loading the missing ones; fns[i] = nullptr where specialization is off.
  void ensure(int device, const std::vector<std::string>& names,
              const std::vector<std::string>& srcs, std::vector<hipFunction_t>& fns) {
    std::lock_guard<std::mutex> lk(mu);
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
      if (!dup && !exists(obj_path(names[i]))) todo.push_back(i);
    }
    if (!todo.empty() && !compile(names, srcs, todo)) return;
    for (size_t i = 0; i < names.size(); ++i) {
      if (fns[i]) continue;
      auto it = loaded.find({device, names[i]});
      if (it == loaded.end()) {
        hipModule_t mod = nullptr;
        hipFunction_t fn = nullptr;
        if (hipModuleLoad(&mod, obj_path(names[i]).c_str()) != hipSuccess ||
            hipModuleGetFunction(&fn, mod, names[i].c_str()) != hipSuccess) {
          (void)hipGetLastError();
          disable("cannot load " + obj_path(names[i]));
          fns.assign(names.size(), nullptr);
          return;
        }
        it = loaded.emplace(std::make_pair(device, names[i]), fn).first;
      }
      fns[i] = it->second;
    }
  }
  bool enabled() {
    std::lock_guard<std::mutex> lk(mu);
    return init();
  }
  // compile without loading (host-only test hook): true when every code object exists after
  const char* compile_only(const std::vector<std::string>& names,
                           const std::vector<std::string>& srcs) {
    std::lock_guard<std::mutex> lk(mu);
    if (!init()) return "specialization unavailable (no hipcc or kernel sources)";
    std::vector<size_t> todo;
    for (size_t i = 0; i < names.size(); ++i)
      if (!exists(obj_path(names[i]))) todo.push_back(i);
    if (!todo.empty() && !compile(names, srcs, todo)) return "hipcc failed";
    return nullptr;
  }
  std::string code_object(const std::string& name) const { return obj_path(name); }
  // processes of this job on the node (ranks): the default compile parallelism is shared
  void set_processes(int p) {
    std::lock_guard<std::mutex> lk(mu);
    procs = std::max(procs, p);
  }

 private:
  std::mutex mu;
  std::map<std::pair<int, std::string>, hipFunction_t> loaded;
  std::string hipcc, csrc, inc, dir;
  int state = 0;  // 0 unknown, 1 on, -1 off
  int procs = 1;
  static bool exists(const std::string& p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0;
  }
  std::string obj_path(const std::string& name) const { return dir + "/" + name + ".hsaco"; }
  void disable(const std::string& why) {
    if (state != -1) fprintf(stderr, "qdc: specialized passes off (%s)\n", why.c_str());
    state = -1;
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
    const char* d = getenv("QDC_JIT_DIR");
    dir = d ? d : "/tmp/qdc_jit_" + std::to_string((unsigned)getuid());
    mkdir(dir.c_str(), 0700);
    if (!exists(csrc + "/qdc_spec.hpp") || access(hipcc.c_str(), X_OK) != 0 || !exists(dir)) {
      disable("no hipcc or kernel sources next to the library");
      return false;
    }
    state = 1;
    return true;
  }
  // the library's own compile-time switches, so the kernels agree with it
  static std::string defines() {
    char b[512];
    snprintf(b, sizeof b,
             "-DQDC_DYN_TAIL=%d -DQDC_FMAX_OPS=%d -DQDC_FMAX_GRAD_RQ=%d -DQDC_RQ_PF_WAVES=%d "
             "-DQDC_RW_WAVES=%d -DQDC_RW_WAVES_ONE=%d -DQDC_RQ_ABL=%d -DQDC_RQ_GSPLIT=%d%s",
             (int)QDC_DYN_TAIL, (int)FMAX_OPS, (int)FMAX_GRAD_RQ, (int)QDC_RQ_PF_WAVES,
             (int)QDC_RW_WAVES, (int)QDC_RW_WAVES_ONE, (int)QDC_RQ_ABL, (int)QDC_RQ_GSPLIT,
             sizeof(real) == 8 ? " -DQDC_F64" : "");
    return b;
  }
  bool compile(const std::vector<std::string>& names, const std::vector<std::string>& srcs,
               const std::vector<size_t>& todo) {
    int jobs = std::min((int)std::thread::hardware_concurrency(), 16) / procs;
    if (const char* e = getenv("QDC_JIT_JOBS")) jobs = atoi(e);
    jobs = std::max(1, std::min(jobs, 16));
    struct Job {
      pid_t pid;
      size_t i;
      std::string tmp;
    };
    std::vector<Job> run;
    size_t next = 0;
    bool ok = true;
    const std::string tag = std::to_string((long)getpid());
    auto reap = [&]() {
      int status = 0;
      const pid_t p = waitpid(run.front().pid, &status, 0);
      Job j = run.front();
      run.erase(run.begin());
      const std::string obj = obj_path(names[j.i]);
      if (p < 0 || !WIFEXITED(status) || WEXITSTATUS(status) != 0 || rename(j.tmp.c_str(), obj.c_str()) != 0) {
        ok = false;
        unlink(j.tmp.c_str());
      }
    };
    while (next < todo.size() || !run.empty()) {
      if (ok && next < todo.size() && (int)run.size() < jobs) {
        const size_t i = todo[next++];
        const std::string src = dir + "/" + names[i] + "." + tag + ".hip";
        FILE* fp = fopen(src.c_str(), "w");
        if (!fp) {
          ok = false;
          continue;
        }
        fputs(srcs[i].c_str(), fp);
        fclose(fp);
        Job j{0, i, obj_path(names[i]) + "." + tag};
        std::vector<std::string> args = {hipcc, "--genco", "-O3", "-std=c++17", "--offload-arch=gfx950",
                                         "-I" + inc, "-I" + csrc, "-o", j.tmp, src};
        {
          std::string d = defines();
          size_t p = 0;
          while (p < d.size()) {
            size_t q = d.find(' ', p);
            if (q == std::string::npos) q = d.size();
            args.insert(args.begin() + 5, d.substr(p, q - p));
            p = q + 1;
          }
        }
        std::vector<char*> argv;
        for (auto& a : args) argv.push_back(const_cast<char*>(a.c_str()));
        argv.push_back(nullptr);
        posix_spawn_file_actions_t fa;
        posix_spawn_file_actions_init(&fa);
        const std::string log = src + ".log";
        posix_spawn_file_actions_addopen(&fa, 1, log.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0600);
        posix_spawn_file_actions_adddup2(&fa, 1, 2);
        const int rc = posix_spawn(&j.pid, hipcc.c_str(), &fa, nullptr, argv.data(), environ);
        posix_spawn_file_actions_destroy(&fa);
        if (rc != 0) {
          ok = false;
          continue;
        }
        run.push_back(j);
        continue;
      }
      if (!run.empty()) reap();
      else break;
    }
    if (!ok) disable("hipcc failed on a pass kernel (sources and logs in " + dir + ")");
    return ok;
  }
};

}  // namespace qdc
