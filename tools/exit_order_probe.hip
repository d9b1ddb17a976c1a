// exit_order_probe.hip — in what order does process exit run the HIP
// runtime's teardown and an exit handler of ours?  (VERDICT r04 next-round 1:
// the r04v child died with SIGSEGV at exit while the doorbell's exit handler
// called hipSetDevice / hipStreamSynchronize from atexit.)
//
// The probe interposes __cxa_atexit and __cxa_thread_atexit_impl (libamdhip64
// imports both) and records every registration with the phase of the program
// it happened in and the library of the callback; each callback is wrapped so
// that, at exit, the order in which the handlers RUN is printed too.  The
// program walks the engine's own sequence: runtime init, an engine stream, four
// call streams, then "the first server" (where engine.cpp registered its exit
// handler), two server streams with a spinning kernel each, eight calling
// threads with thread-local staging — and exits with the servers still
// spinning.  Our handler reports whether the runtime still answers when it
// runs (hipStreamQuery on a server stream) and, with `hip` as argv[1], calls
// hipSetDevice + hipStreamSynchronize as the r04v handler did.
//
// usage: exit_order_probe [hip|nohip]
#include <dlfcn.h>
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

static const char* volatile g_phase = "static-init";
static std::atomic<int> g_reg_seq{0}, g_run_seq{0};

struct Reg {
  void (*f)(void*);
  void* arg;
  int seq;
  const char* phase;
  const char* kind;
  char lib[64];
  char owner[64];
};

static void lib_of(void* p, char* out, size_t n) {
  Dl_info di;
  const char* s = "?";
  if (dladdr(p, &di) && di.dli_fname) {
    s = strrchr(di.dli_fname, '/');
    s = s ? s + 1 : di.dli_fname;
  }
  snprintf(out, n, "%s", s);
}

static void run_wrapped(void* p) {
  Reg* r = static_cast<Reg*>(p);
  const int n = g_run_seq.fetch_add(1);
  fprintf(stderr, "EXIT-RUN #%d %s reg#%d (registered in phase '%s', owner %s)\n", n, r->kind,
          r->seq, r->phase, r->owner);
  r->f(r->arg);
}

static Reg* make_reg(const char* kind, void (*f)(void*), void* arg, void* dso) {
  Reg* r = static_cast<Reg*>(malloc(sizeof(Reg)));
  r->f = f;
  r->arg = arg;
  r->seq = g_reg_seq.fetch_add(1);
  r->phase = g_phase;
  r->kind = kind;
  lib_of((void*)f, r->lib, sizeof(r->lib));
  if (dso) lib_of(dso, r->owner, sizeof(r->owner));
  else snprintf(r->owner, sizeof(r->owner), "-");
  fprintf(stderr, "REG #%d %-10s phase '%s' owner %s fn-in %s\n", r->seq, kind, r->phase,
          r->owner, r->lib);
  return r;
}

extern "C" int __cxa_atexit(void (*f)(void*), void* arg, void* dso) {
  using fn = int (*)(void (*)(void*), void*, void*);
  static fn real = (fn)dlsym(RTLD_NEXT, "__cxa_atexit");
  return real(run_wrapped, make_reg("atexit", f, arg, dso), dso);
}

extern "C" int __cxa_thread_atexit_impl(void (*f)(void*), void* obj, void* dso) {
  using fn = int (*)(void (*)(void*), void*, void*);
  static fn real = (fn)dlsym(RTLD_NEXT, "__cxa_thread_atexit_impl");
  return real(run_wrapped, make_reg("tls-dtor", f, obj, dso), dso);
}

__global__ void spin_kernel(const uint32_t* stop, unsigned long long lifetime) {
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) == 0 &&
         __builtin_amdgcn_s_memrealtime() - t0 < lifetime)
    __builtin_amdgcn_s_sleep(8);
}
__global__ void touch_kernel(uint8_t* p) { p[threadIdx.x] ^= 1; }

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));            \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

static bool g_hip_in_handler = false;
static hipStream_t g_srv[2];
static uint32_t* g_stop = nullptr;

static void our_exit_handler() {
  fprintf(stderr, "OUR-HANDLER runs (run order #%d)\n", g_run_seq.load());
  __atomic_store_n(g_stop, 1u, __ATOMIC_RELEASE);
  const hipError_t q = hipStreamQuery(g_srv[0]);
  fprintf(stderr, "OUR-HANDLER hipStreamQuery(server 0) = %d (%s)\n", (int)q,
          q == hipSuccess ? "idle" : q == hipErrorNotReady ? "busy" : "error");
  if (g_hip_in_handler) {
    for (hipStream_t s : g_srv) {
      const hipError_t a = hipSetDevice(0), b = hipStreamSynchronize(s);
      fprintf(stderr, "OUR-HANDLER hipSetDevice %d hipStreamSynchronize %d\n", (int)a, (int)b);
    }
  }
}

struct Staging {  // engine.cpp's thread-local staging, in miniature
  uint8_t* d = nullptr;
  uint8_t* h = nullptr;
  hipEvent_t ev = nullptr;
  ~Staging() {
    if (d) (void)hipFree(d);
    if (h) (void)hipHostFree(h);
    if (ev) (void)hipEventDestroy(ev);
  }
};
static thread_local Staging t_stage;

__attribute__((destructor)) static void probe_fini() {
  fprintf(stderr, "LIB-DESTRUCTOR (DT_FINI_ARRAY) runs after %d exit handlers\n",
          g_run_seq.load());
}

int main(int argc, char** argv) {
  g_hip_in_handler = argc > 1 && !strcmp(argv[1], "hip");
  g_phase = "hipGetDeviceCount";
  int n = 0;
  CK(hipGetDeviceCount(&n));
  g_phase = "hipSetDevice";
  CK(hipSetDevice(0));
  g_phase = "engine stream + buffers";
  hipStream_t es;
  CK(hipStreamCreateWithFlags(&es, hipStreamNonBlocking));
  uint8_t* d = nullptr;
  CK(hipMalloc(&d, 1 << 20));
  uint8_t* h = nullptr;
  CK(hipHostMalloc((void**)&h, 1 << 20, hipHostMallocDefault));
  hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(64), 0, es, d);
  CK(hipStreamSynchronize(es));
  g_phase = "4 call streams";
  hipStream_t cs[4];
  for (auto& s : cs) {
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(64), 0, s, d);
    CK(hipStreamSynchronize(s));
  }
  g_phase = "first server: our atexit";
  atexit(our_exit_handler);
  g_phase = "server streams + spin kernels";
  CK(hipHostMalloc((void**)&g_stop, 4096, hipHostMallocDefault));
  memset(g_stop, 0, 4096);
  uint32_t* d_stop = nullptr;
  CK(hipHostGetDevicePointer((void**)&d_stop, g_stop, 0));
  for (auto& s : g_srv) {
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipLaunchKernelGGL(spin_kernel, dim3(1), dim3(64), 0, s, d_stop, 500000000ull);  // 5 s max
  }
  g_phase = "8 calling threads";
  std::vector<std::thread> th;
  for (int t = 0; t < 8; t++)
    th.emplace_back([&cs, t] {
      CK(hipSetDevice(0));
      CK(hipMalloc(&t_stage.d, 1 << 20));
      CK(hipHostMalloc((void**)&t_stage.h, 1 << 20, hipHostMallocDefault));
      CK(hipEventCreateWithFlags(&t_stage.ev, hipEventDisableTiming));
      hipLaunchKernelGGL(touch_kernel, dim3(1), dim3(64), 0, cs[t % 4], t_stage.d);
      CK(hipEventRecord(t_stage.ev, cs[t % 4]));
      CK(hipEventSynchronize(t_stage.ev));
    });
  for (auto& t : th) t.join();
  g_phase = "after threads";
  fprintf(stderr, "MAIN returns (servers still spinning); %d registrations\n", g_reg_seq.load());
  return 0;
}
