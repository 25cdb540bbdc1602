// cold_probe.cpp -- diagnostic: why a fresh process's first HIP stream can
// take ~160 ms (bench.py's "cold" end-to-end leg) while the next fresh
// process takes ~20 ms.  Two roles, run as separate processes:
//
//   cold_probe hold GB [free|exit]   allocate GB GiB of device memory, write it
//                                    (hipMemset), then hipFree it before exit
//                                    ("free") or just exit ("exit")
//   cold_probe probe                 a fresh process's HIP start-up, step by
//                                    step: runtime init (device count), device
//                                    memory info, the first stream (the first
//                                    call that builds the device context), a
//                                    second stream, a 64 MiB hipMalloc, a
//                                    64 MiB pinned host buffer
//
// tools/probe/cold_probe.sh runs "hold X; probe; probe; sleep; probe" for
// several X, so the first stream's cost can be read against the device
// memory the previous process held and how long ago it exited.
// Build: hipcc -O2 -o tools/probe/cold_probe tools/probe/cold_probe.cpp
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <chrono>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char **argv) {
  if (argc >= 3 && strcmp(argv[1], "hold") == 0) {
    const size_t gb = strtoull(argv[2], NULL, 0);
    const bool do_free = argc < 4 || strcmp(argv[3], "exit") != 0;
    double t0 = now();
    void *p = nullptr;
    if (gb > 0) {
      if (hipMalloc(&p, gb << 30) != hipSuccess || hipMemset(p, 0x5a, gb << 30) != hipSuccess ||
          hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "hold %zu GiB failed\n", gb);
        return 1;
      }
    }
    const double ta = now() - t0;
    t0 = now();
    if (p && do_free) (void) hipFree(p);
    printf("{\"role\":\"hold\",\"gib\":%zu,\"alloc_memset_ms\":%.2f,\"free_ms\":%.2f,\"freed_before_exit\":%s}\n",
           gb, ta * 1e3, (now() - t0) * 1e3, do_free ? "true" : "false");
    return 0;
  }
  double t0 = now(), t;
  int n = 0;
  (void) hipGetDeviceCount(&n);
  const double t_init = now() - t0;
  t0 = now();
  (void) hipSetDevice(0);
  const double t_set = now() - t0;
  size_t fr = 0, tot = 0;
  t0 = now();
  (void) hipMemGetInfo(&fr, &tot);
  const double t_info = now() - t0;
  hipStream_t s1, s2;
  t0 = now();
  (void) hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  const double t_s1 = now() - t0;
  t0 = now();
  (void) hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  const double t_s2 = now() - t0;
  size_t fr2 = 0, tot2 = 0;
  (void) hipMemGetInfo(&fr2, &tot2);
  void *d = nullptr, *h = nullptr;
  t0 = now();
  (void) hipMalloc(&d, 64u << 20);
  const double t_m = now() - t0;
  t0 = now();
  (void) hipHostMalloc(&h, 64u << 20, hipHostMallocDefault);
  const double t_h = now() - t0;
  t = now();
  (void) hipMemsetAsync(d, 0, 64u << 20, s1);
  (void) hipStreamSynchronize(s1);
  const double t_first_op = now() - t;
  printf("{\"role\":\"probe\",\"init_ms\":%.2f,\"set_device_ms\":%.2f,\"mem_info_ms\":%.2f,"
         "\"free_gib_before_stream\":%.1f,\"total_gib\":%.1f,\"first_stream_ms\":%.2f,"
         "\"second_stream_ms\":%.2f,\"free_gib_after_stream\":%.1f,\"malloc64m_ms\":%.2f,"
         "\"hostmalloc64m_ms\":%.2f,\"first_memset_sync_ms\":%.2f}\n",
         t_init * 1e3, t_set * 1e3, t_info * 1e3, fr / 1073741824.0, tot / 1073741824.0, t_s1 * 1e3,
         t_s2 * 1e3, fr2 / 1073741824.0, t_m * 1e3, t_h * 1e3, t_first_op * 1e3);
  return 0;
}
