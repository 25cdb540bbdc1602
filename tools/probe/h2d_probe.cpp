// h2d_probe.cpp -- diagnostic: is a first call's H2D slower because the
// destination is freshly allocated device memory?  Times 64 MiB pinned ->
// device copies over a fresh 3 GiB allocation (first pass), the same region
// again (second pass), and a second fresh allocation that was memset first.
// Build: hipcc -O2 -o tools/probe/h2d_probe tools/probe/h2d_probe.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#include <chrono>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CHK(x)                                                                       \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                        \
      return 1;                                                                      \
    }                                                                                \
  } while (0)

static int pass(const char *name, char *dst, size_t total, void *pin, size_t chunk, hipStream_t s) {
  const double t0 = now();
  for (size_t off = 0; off < total; off += chunk) {
    const size_t n = total - off < chunk ? total - off : chunk;
    CHK(hipMemcpyAsync(dst + off, pin, n, hipMemcpyHostToDevice, s));
  }
  CHK(hipStreamSynchronize(s));
  const double dt = now() - t0;
  printf("%-34s %7.2f ms  %6.1f GB/s\n", name, dt * 1e3, total / dt / 1e9);
  return 0;
}

int main() {
  const size_t total = 3ull << 30, chunk = 64ull << 20;
  hipStream_t s;
  CHK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  void *pin = nullptr;
  CHK(hipHostMalloc(&pin, chunk, hipHostMallocDefault));
  memset(pin, 7, chunk);
  char *a = nullptr, *b = nullptr, *c = nullptr;
  double t0 = now();
  CHK(hipMalloc(&a, total));
  printf("hipMalloc 3 GiB: %.2f ms\n", (now() - t0) * 1e3);
  if (pass("fresh allocation, first pass", a, total, pin, chunk, s)) return 1;
  if (pass("same allocation, second pass", a, total, pin, chunk, s)) return 1;
  CHK(hipMalloc(&b, total));
  t0 = now();
  CHK(hipMemsetAsync(b, 0, total, s));
  CHK(hipStreamSynchronize(s));
  printf("memset of a fresh 3 GiB: %.2f ms\n", (now() - t0) * 1e3);
  if (pass("fresh allocation after memset", b, total, pin, chunk, s)) return 1;
  CHK(hipFree(a));
  CHK(hipMalloc(&c, total));
  if (pass("re-allocated (freed 3 GiB reused)", c, total, pin, chunk, s)) return 1;
  CHK(hipFree(b));
  CHK(hipFree(c));
  CHK(hipHostFree(pin));
  return 0;
}
