// pin_probe.cpp -- diagnostic: what a first call's pinned staging ring costs
// on this box (hipHostMalloc of 16..128 MiB, cold and warm; hipHostRegister
// of an already-touched malloc block; the thread spawns of a staging fill).
// Build: hipcc -O2 -o tools/probe/pin_probe tools/probe/pin_probe.cpp -lpthread
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>
#include <thread>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  double t0 = now();
  int n = 0;
  (void) hipGetDeviceCount(&n);
  printf("hip init + device count: %.1f ms (%d devices)\n", (now() - t0) * 1e3, n);
  t0 = now();
  hipStream_t s;
  (void) hipStreamCreate(&s);
  printf("stream create: %.2f ms\n", (now() - t0) * 1e3);
  for (size_t mb : {16, 32, 64, 128, 64}) {
    void *p = nullptr;
    t0 = now();
    hipError_t e = hipHostMalloc(&p, mb << 20, hipHostMallocDefault);
    const double ta = now() - t0;
    t0 = now();
    (void) hipHostFree(p);
    printf("hipHostMalloc %3zu MiB: %7.2f ms (free %.2f ms) %s\n", mb, ta * 1e3, (now() - t0) * 1e3,
           e == hipSuccess ? "" : "FAILED");
  }
  for (size_t mb : {16, 64}) {
    char *q = (char *) aligned_alloc(2 << 20, mb << 20);
    memset(q, 1, mb << 20);
    t0 = now();
    hipError_t e = hipHostRegister(q, mb << 20, hipHostRegisterDefault);
    const double tr = now() - t0;
    t0 = now();
    (void) hipHostUnregister(q);
    printf("hipHostRegister %3zu MiB (touched): %7.2f ms (unregister %.2f ms) %s\n", mb, tr * 1e3,
           (now() - t0) * 1e3, e == hipSuccess ? "" : "FAILED");
    free(q);
  }
  // thread spawn + join cost of one 12-thread fill
  t0 = now();
  for (int k = 0; k < 50; k++) {
    std::vector<std::thread> th;
    for (int t = 0; t < 11; t++) th.emplace_back([] {});
    for (auto &x : th) x.join();
  }
  printf("11-thread spawn+join: %.1f us each\n", (now() - t0) * 1e6 / 50);
  void *d = nullptr;
  for (size_t gb : {1, 3}) {
    t0 = now();
    (void) hipMalloc(&d, gb << 30);
    const double tm = now() - t0;
    t0 = now();
    (void) hipFree(d);
    printf("hipMalloc %zu GiB: %.2f ms (free %.2f ms)\n", gb, tm * 1e3, (now() - t0) * 1e3);
  }
  return 0;
}
