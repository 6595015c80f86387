// Probe: do concurrent host threads, each with its own stream, scale their small-call round trips?
// Each "call" = [2 KiB pinned->device copy] + a 1568-workgroup kernel + [a 31-workgroup kernel] +
// stream sync, the shape of a search scoring call (upload blit, interpreter, partial reduce).
// Aggregate calls/s for 1..8 threads and three call shapes: is the device's dispatch path shared?
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <thread>
#include <vector>

__global__ void k_work(const unsigned* p, unsigned* out, int spin) {
  unsigned s = p[threadIdx.x & 511];
  for (int i = 0; i < spin; ++i) s = s * 1664525u + 1013904223u;
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}
__global__ void k_small(const unsigned* in, unsigned* out) {
  if (threadIdx.x == 0) out[blockIdx.x] = in[blockIdx.x] + 1;
}

int main() {
  const int reps = 2000;
  for (int shape = 0; shape < 3; ++shape) {
    const char* nm = shape == 0 ? "copy + kernel + kernel" : shape == 1 ? "kernel + kernel" : "kernel";
    for (int T : {1, 2, 4, 6, 8}) {
      std::vector<std::thread> th;
      std::atomic<int> ready{0};
      std::atomic<bool> go{false};
      std::vector<double> secs(T);
      for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
          hipStream_t s;
          (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
          unsigned *d, *o, *h;
          (void)hipMalloc(&d, 4096);
          (void)hipMalloc(&o, 4 * 2048);
          (void)hipHostMalloc((void**)&h, 4096, hipHostMallocDefault);
          for (int i = 0; i < 1024; ++i) h[i] = i;
          auto call = [&] {
            if (shape == 0) (void)hipMemcpyAsync(d, h, 2048, hipMemcpyHostToDevice, s);
            k_work<<<1568, 256, 0, s>>>(d, o, 64);
            if (shape <= 1) k_small<<<31, 64, 0, s>>>(o, o + 1600);
            (void)hipStreamSynchronize(s);
          };
          for (int i = 0; i < 100; ++i) call();
          ready++;
          while (!go.load()) {}
          auto t0 = std::chrono::steady_clock::now();
          for (int i = 0; i < reps; ++i) call();
          secs[t] = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
          (void)hipStreamSynchronize(s);
          (void)hipFree(d);
          (void)hipFree(o);
          (void)hipHostFree(h);
          (void)hipStreamDestroy(s);
        });
      while (ready.load() < T) {}
      go = true;
      for (auto& x : th) x.join();
      double mx = 0;
      for (double v : secs) mx = v > mx ? v : mx;
      std::printf("%-24s threads %d: %8.0f calls/s aggregate, %6.2f us per call per thread\n", nm, T,
                  T * reps / mx, mx / reps * 1e6);
      std::fflush(stdout);
    }
  }
  std::printf("done\n");
  return 0;
}
