// Probe: can the host write a small call's programs straight into device memory (no upload blit)?
// For fine-grained / uncached device allocations and managed memory: pointer attributes (a host
// mapping?), then, only where the runtime reports one, the latency of host memcpy + launch + sync
// against a pinned->device hipMemcpyAsync + launch + sync (the current path) and a launch alone.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <atomic>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void k_ptr(const unsigned* p, int n, unsigned* out) {
  unsigned s = 0;
  for (int i = threadIdx.x; i < n; i += blockDim.x) s += p[i] * (i + 1u);
  if (threadIdx.x == 0) out[blockIdx.x] = s;
}

int main() {
  const int n = 1024, bytes = n * 4;  // 4 KiB
  const int blocks = 1568;
  unsigned* out; unsigned* dbuf; unsigned* hbuf;
  CK(hipMalloc(&out, blocks * 4)); CK(hipMalloc(&dbuf, bytes));
  CK(hipHostMalloc((void**)&hbuf, bytes, hipHostMallocDefault));
  for (int i = 0; i < n; ++i) hbuf[i] = i * 2654435761u;
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  struct Cand { const char* name; void* p; };
  Cand c[3] = {{"fine-grained device", nullptr}, {"uncached device", nullptr}, {"managed", nullptr}};
  hipError_t e0 = hipExtMallocWithFlags(&c[0].p, bytes, hipDeviceMallocFinegrained);
  hipError_t e1 = hipExtMallocWithFlags(&c[1].p, bytes, hipDeviceMallocUncached);
  hipError_t e2 = hipMallocManaged(&c[2].p, bytes);
  std::printf("alloc rc %d %d %d\n", int(e0), int(e1), int(e2));
  (void)hipGetLastError();
  void* host_ok[3] = {nullptr, nullptr, nullptr};
  for (int k = 0; k < 3; ++k) {
    if (!c[k].p) continue;
    hipPointerAttribute_t at{};
    hipError_t pe = hipPointerGetAttributes(&at, c[k].p);
    std::printf("%-22s p=%p attr rc %d type %d device %d hostPointer %p devicePointer %p isManaged %d\n", c[k].name, c[k].p,
                int(pe), int(at.type), at.device, at.hostPointer, at.devicePointer, int(at.isManaged));
    (void)hipGetLastError();
    if (pe == hipSuccess && at.hostPointer) host_ok[k] = at.hostPointer;
  }
  auto bench = [&](const char* name, auto fn) {
    for (int i = 0; i < 200; ++i) fn();
    const int reps = 3000;
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) fn();
    auto t1 = std::chrono::steady_clock::now();
    std::printf("%-48s %8.2f us per call\n", name, std::chrono::duration<double, std::micro>(t1 - t0).count() / reps);
  };
  for (int b : {blocks, 64}) {
    std::printf("-- %d workgroups\n", b);
    bench("(b) 4 KiB blit + launch + sync", [&] {
      (void)hipMemcpyAsync(dbuf, hbuf, bytes, hipMemcpyHostToDevice, s);
      k_ptr<<<b, 256, 0, s>>>(dbuf, n, out); (void)hipStreamSynchronize(s); });
    bench("(c) launch + sync", [&] { k_ptr<<<b, 256, 0, s>>>(dbuf, n, out); (void)hipStreamSynchronize(s); });
    for (int k = 0; k < 3; ++k) {
      if (!host_ok[k]) continue;
      char nm[96];
      std::snprintf(nm, sizeof nm, "(e) host memcpy into %s + launch + sync", c[k].name);
      unsigned* dp = static_cast<unsigned*>(c[k].p);
      unsigned* hp = static_cast<unsigned*>(host_ok[k]);
      bench(nm, [&] {
        std::memcpy(hp, hbuf, bytes);
        std::atomic_thread_fence(std::memory_order_seq_cst);
        k_ptr<<<b, 256, 0, s>>>(dp, n, out); (void)hipStreamSynchronize(s); });
      // correctness of what the kernel saw
      unsigned got[1] = {0};
      (void)hipMemcpy(got, out, 4, hipMemcpyDeviceToHost);
      unsigned ref = 0;
      for (int i = 0; i < n; i += 256) {}
      for (int i = 0; i < n; i += 256) ref += hbuf[i] * (i + 1u);
      std::printf("   block 0 thread-0 partial %u expected %u %s\n", got[0], ref, got[0] == ref ? "OK" : "MISMATCH");
    }
  }
  CK(hipStreamSynchronize(s));
  std::printf("done\n");
  return 0;
}
