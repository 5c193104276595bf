// qdc_jit.hpp — the specialized reverse-pass kernels (qdc_spec.hpp): source per pass program,
// compiled with hipcc for gfx950 on first use, cached on disk and per device.
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

// Source of one pass program: steps as emitted into the program (relayouts with the layouts
// before and after, stages with their fop), in order.
struct SpecStep {
  bool relayout;
  RqLayout Lc, Ln;  // relayout: current and new layout
  fop F;            // stage: kind (+ FOP_GAMMA), slot case in t1
};
inline std::string spec_program_source(const std::vector<SpecStep>& steps, uint32_t T) {
  std::string b;
  char tmp[512];
  uint32_t ri = 0;
  auto arr = [&](const uint32_t* v, int n) {
    std::string s = "{";
    for (int i = 0; i < n; ++i) {
      snprintf(tmp, sizeof tmp, "%s%uu", i ? "," : "", v[i]);
      s += tmp;
    }
    return s + "}";
  };
  for (size_t j = 0; j < steps.size(); ++j) {
    const SpecStep& s = steps[j];
    if (s.relayout) {
      const rq_layout c = rq_descriptor(s.Lc, T), n = rq_descriptor(s.Ln, T);
      b += "    { constexpr uint32_t rc[32] = " + arr(c.rp, 32) + ", tc[8] = " + arr(c.tv, 8) +
           ", rn[32] = " + arr(n.rp, 32) + ", tn[8] = " + arr(n.tv, 8) +
           ";\n      spec_xchg(xf, E, rc, tc, rn, tn); spec_xchg(xb, E, rc, tc, rn, tn); }\n";
      continue;
    }
    const uint32_t kind = s.F.kind & 7u;
    const bool gamma = (s.F.kind & FOP_GAMMA) != 0;
    const uint32_t c = s.F.t1;
    if (kind == FK_Q1)
      snprintf(tmp, sizeof tmp, "    rq_q1<%u, true, 32>(xf, xb, E.mats + E.ops[%zu].mat, %s, &E.accw[%u][0]);\n",
               c, j, gamma ? "true" : "false", ri);
    else
      snprintf(tmp, sizeof tmp, "    %s<%u, %u, true, 32>(xf, xb, E.mats + E.ops[%zu].mat, %s, &E.accw[%u][0]);\n",
               kind == FK_DIAG ? "rq_diag" : "rq_q2", c >> 3, c & 7u, j, gamma ? "true" : "false", ri);
    b += tmp;
    if (gamma) ++ri;
  }
  return b;
}
inline std::string spec_kernel_source(const std::string& name, const std::string& body) {
  return "#include \"qdc_spec.hpp\"\n"
         "namespace {\n"
         "struct Prog {\n"
         "  __device__ __forceinline__ void operator()(qdc::cx (&xf)[32], qdc::cx (&xb)[32],\n"
         "                                             const qdc::SpecEnv& E) const {\n"
         "    using namespace qdc;\n" +
         body +
         "  }\n"
         "};\n"
         "}  // namespace\n"
         "extern \"C\" __global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2, 2)))\n"
         "void " + name + "(qdc::chunk* __restrict__ f, qdc::chunk* __restrict__ b,\n"
         "    const qdc::fop* __restrict__ ops, const qdc::cx* __restrict__ mats, qdc::fgeo fg,\n"
         "    uint32_t l0, qdc::cx* __restrict__ partials, uint64_t slot_stride) {\n"
         "  qdc::rw_spec_two<Prog>(f, b, ops, mats, fg, l0, partials, slot_stride);\n"
         "}\n";
}

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

 private:
  std::mutex mu;
  std::map<std::pair<int, std::string>, hipFunction_t> loaded;
  std::string hipcc, csrc, inc, dir;
  int state = 0;  // 0 unknown, 1 on, -1 off
  static bool exists(const std::string& p) {
    struct stat st;
    return stat(p.c_str(), &st) == 0;
  }
  std::string obj_path(const std::string& name) const { return dir + "/" + name + ".hsaco"; }
  void disable(const std::string& why) {
    if (state != -1) fprintf(stderr, "qdc: specialized reverse passes off (%s)\n", why.c_str());
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
    char b[256];
    snprintf(b, sizeof b, "-DQDC_DYN_TAIL=%d -DQDC_FMAX_OPS=%d -DQDC_FMAX_GRAD_RQ=%d", (int)QDC_DYN_TAIL,
             (int)FMAX_OPS, (int)FMAX_GRAD_RQ);
    return b;
  }
  bool compile(const std::vector<std::string>& names, const std::vector<std::string>& srcs,
               const std::vector<size_t>& todo) {
    int jobs = (int)std::thread::hardware_concurrency();
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
