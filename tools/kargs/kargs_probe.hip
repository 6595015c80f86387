// Probe: can a launch carry a small call's programs in its kernel arguments (no upload blit)?
// Checks the bytes arrive, where the kernarg segment lives, and the launch+sync latency of
// (a) 4 KiB by-value arguments, (b) a 4 KiB pinned->device hipMemcpyAsync then a small-argument
// launch (the current path), (c) a small-argument launch alone.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

struct alignas(16) Inline { unsigned char b[4096]; };

__global__ void k_inline(Inline in, int n, unsigned* out, unsigned long long* addr) {
  const unsigned char* p = in.b;
  unsigned s = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i] * (i + 1u);
  atomicAdd(out, s);
  if (threadIdx.x == 0 && blockIdx.x == 0) addr[0] = (unsigned long long)(const void*)p;
}
__global__ void k_ptr(const unsigned char* p, int n, unsigned* out) {
  unsigned s = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i] * (i + 1u);
  atomicAdd(out, s);
}

int main() {
  const int n = 4096;
  Inline in;
  unsigned ref = 0;
  for (int i = 0; i < n; ++i) { in.b[i] = (unsigned char)(i * 7 + 3); ref += in.b[i] * (i + 1u); }
  unsigned* out; unsigned long long* addr; unsigned char* dbuf; unsigned char* hbuf;
  CK(hipMalloc(&out, 4)); CK(hipMalloc(&addr, 8)); CK(hipMalloc(&dbuf, n));
  CK(hipHostMalloc((void**)&hbuf, n, hipHostMallocDefault));
  std::memcpy(hbuf, in.b, n);
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int blocks = 1568;
  // correctness
  CK(hipMemsetAsync(out, 0, 4, s));
  k_inline<<<blocks, 256, 0, s>>>(in, n, out, addr);
  CK(hipGetLastError());
  unsigned got = 0; unsigned long long a = 0;
  CK(hipMemcpyAsync(&got, out, 4, hipMemcpyDeviceToHost, s));
  CK(hipMemcpyAsync(&a, addr, 8, hipMemcpyDeviceToHost, s));
  CK(hipStreamSynchronize(s));
  hipPointerAttribute_t at{};
  hipError_t pe = hipPointerGetAttributes(&at, (void*)a);
  std::printf("inline sum %u expected %u (x%d blocks: %u) %s; kernarg at 0x%llx: attr rc %d type %d device %d\n",
              got, ref * blocks, blocks, ref * blocks, got == ref * blocks ? "OK" : "MISMATCH", a, int(pe),
              pe == hipSuccess ? int(at.type) : -1, pe == hipSuccess ? at.device : -1);
  (void)hipGetLastError();
  auto bench = [&](const char* name, auto fn) {
    for (int i = 0; i < 200; ++i) fn();
    const int reps = 3000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) fn();
    auto t1 = std::chrono::steady_clock::now();
    std::printf("%-44s %8.2f us per launch+sync\n", name, std::chrono::duration<double, std::micro>(t1 - t0).count() / reps);
  };
  for (int b : {1568, 64}) {
    std::printf("-- %d workgroups\n", b);
    bench("(a) 4 KiB inline arguments", [&] { k_inline<<<b, 256, 0, s>>>(in, n, out, addr); (void)hipStreamSynchronize(s); });
    bench("(b) 4 KiB blit + pointer argument", [&] {
      (void)hipMemcpyAsync(dbuf, hbuf, n, hipMemcpyHostToDevice, s);
      k_ptr<<<b, 256, 0, s>>>(dbuf, n, out); (void)hipStreamSynchronize(s); });
    bench("(c) pointer argument only", [&] { k_ptr<<<b, 256, 0, s>>>(dbuf, n, out); (void)hipStreamSynchronize(s); });
    bench("(d) pinned host pointer argument", [&] { k_ptr<<<b, 256, 0, s>>>(hbuf, n, out); (void)hipStreamSynchronize(s); });
  }
  CK(hipStreamSynchronize(s));
  std::printf("done\n");
  return 0;
}
