// Probe: round-trip latency of a small scoring-shaped call served by a PERSISTENT kernel (resident
// workgroups that poll a doorbell in pinned host memory) against the launch path (upload copy +
// work kernel + reduce kernel + stream sync).  The work is the same in both: every workgroup reads
// a 1 KiB "program" from the host side of the call, folds its slice of a device-resident array
// scaled by it, and the partial sums are reduced to one value the host reads.
//
// Polls are relaxed loads (no cache invalidation per poll); one acquire fence follows a new value.
//
// Termination: every wave reaches its exit. A workgroup leaves the poll loop on a new doorbell, on
// the host's stop word, or after max_idle polls with no new call (bounded sleep per poll), so the
// grid drains within ~max_idle x sleep after the last call even if the host goes away. The host
// waits for each call's done word with a wall-clock time-out and then stops the kernel.
#include <hip/hip_runtime.h>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

constexpr int kProgWords = 256;  // 1 KiB
constexpr uint32_t kQuit = 0xffffffffu;

struct Mailbox {               // pinned host memory, one 64-byte line per field
  uint32_t doorbell; uint32_t p0[15];
  uint32_t done;     uint32_t p1[15];
  uint32_t stop;     uint32_t p2[15];
  float result;      uint32_t p3[15];
  uint32_t prog[kProgWords];
};

__device__ inline float fold_slice(const float* __restrict__ data, int n, int nb, int b, float scale) {
  const int per = (n + nb - 1) / nb;
  const int lo = b * per, hi = lo + per < n ? lo + per : n;
  float s = 0.0f;
  for (int i = lo + int(threadIdx.x); i < hi; i += int(blockDim.x)) s += data[i] * scale;
  // block sum through LDS
  __shared__ float red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int h = int(blockDim.x) / 2; h > 0; h >>= 1) {
    if (int(threadIdx.x) < h) red[threadIdx.x] += red[threadIdx.x + h];
    __syncthreads();
  }
  return red[0];
}

__global__ void __launch_bounds__(256) k_persist(Mailbox* mb, const float* data, int n, float* partial,
                                                 uint32_t* count, int max_idle) {
  __shared__ uint32_t s_seq;
  __shared__ float s_scale;
  uint32_t last = 0;
  for (;;) {
    if (threadIdx.x == 0) {
      uint32_t seq = kQuit;
      for (int polls = 0; polls < max_idle; ++polls) {
        const uint32_t d = __hip_atomic_load(&mb->doorbell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        if (d != last) { seq = d; __atomic_thread_fence(__ATOMIC_ACQUIRE); break; }
        if (__hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
        __builtin_amdgcn_s_sleep(1);
      }
      s_seq = seq;
    }
    __syncthreads();
    const uint32_t seq = s_seq;
    if (seq == kQuit) return;  // (every thread of the block: s_seq is block-uniform)
    last = seq;
    // the call's program: one word per thread from host memory
    const uint32_t w = __hip_atomic_load(&mb->prog[threadIdx.x % kProgWords], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    if (threadIdx.x == 0) s_scale = float(w & 0xffu) / 255.0f;
    __syncthreads();
    const float s = fold_slice(data, n, int(gridDim.x), int(blockIdx.x), s_scale);
    if (threadIdx.x == 0) {
      partial[blockIdx.x] = s;
      __threadfence();  // the partial before the count (agent scope)
      const uint32_t prev = atomicAdd(count, 1u);
      if (prev + 1u == seq * gridDim.x) {  // the call's last block: reduce, answer the host
        __threadfence();
        float t = 0.0f;
        for (unsigned b = 0; b < gridDim.x; ++b) t += __hip_atomic_load(&partial[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&mb->result, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->done, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();
  }
}

// Variant 2: only workgroup 0 talks to the host. It polls the host doorbell, copies the call's
// program into device memory and publishes a device doorbell (agent scope); the other workgroups poll
// that device word instead of host memory.
__global__ void __launch_bounds__(256) k_persist2(Mailbox* mb, const float* data, int n, float* partial,
                                                  uint32_t* count, uint32_t* dprog, uint32_t* ddoor, int max_idle) {
  __shared__ uint32_t s_seq;
  __shared__ float s_scale;
  uint32_t last = 0;
  for (;;) {
    if (blockIdx.x == 0) {
      if (threadIdx.x == 0) {
        uint32_t seq = kQuit;
        for (int polls = 0; polls < max_idle; ++polls) {
          const uint32_t d = __hip_atomic_load(&mb->doorbell, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
          if (d != last) { seq = d; __atomic_thread_fence(__ATOMIC_ACQUIRE); break; }
          if (__hip_atomic_load(&mb->stop, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM)) break;
          __builtin_amdgcn_s_sleep(1);
        }
        s_seq = seq;
      }
      __syncthreads();
      const uint32_t seq = s_seq;
      if (seq != kQuit) {
        const uint32_t w = __hip_atomic_load(&mb->prog[threadIdx.x % kProgWords], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&dprog[threadIdx.x % kProgWords], w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
      __syncthreads();
      if (threadIdx.x == 0) __hip_atomic_store(ddoor, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      if (seq == kQuit) return;
      last = seq;
    } else {
      if (threadIdx.x == 0) {
        uint32_t seq = kQuit;
        for (int polls = 0; polls < 16 * max_idle; ++polls) {
          const uint32_t d = __hip_atomic_load(ddoor, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          if (d != last) { seq = d; __atomic_thread_fence(__ATOMIC_ACQUIRE); break; }
          __builtin_amdgcn_s_sleep(1);
        }
        s_seq = seq;
      }
      __syncthreads();
      const uint32_t seq = s_seq;
      if (seq == kQuit) return;
      last = seq;
    }
    if (threadIdx.x == 0) s_scale = float(__hip_atomic_load(&dprog[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & 0xffu) / 255.0f;
    __syncthreads();
    const float s = fold_slice(data, n, int(gridDim.x), int(blockIdx.x), s_scale);
    if (threadIdx.x == 0) {
      partial[blockIdx.x] = s;
      __threadfence();
      const uint32_t prev = atomicAdd(count, 1u);
      if (prev + 1u == last * gridDim.x) {
        __threadfence();
        float t = 0.0f;
        for (unsigned b = 0; b < gridDim.x; ++b) t += __hip_atomic_load(&partial[b], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(&mb->result, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        __hip_atomic_store(&mb->done, last, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
      }
    }
    __syncthreads();
  }
}

// the launch path's two kernels
__global__ void __launch_bounds__(256) k_work(const uint32_t* prog, const float* data, int n, float* partial) {
  __shared__ float s_scale;
  if (threadIdx.x == 0) s_scale = float(prog[0] & 0xffu) / 255.0f;
  __syncthreads();
  const float s = fold_slice(data, n, int(gridDim.x), int(blockIdx.x), s_scale);
  if (threadIdx.x == 0) partial[blockIdx.x] = s;
}
__global__ void k_reduce(const float* partial, int nb, float* out) {
  if (threadIdx.x == 0) {
    float t = 0.0f;
    for (int b = 0; b < nb; ++b) t += partial[b];
    *out = t;
  }
}

int main() {
  const int n = 100000;
  std::vector<float> h(n);
  for (int i = 0; i < n; ++i) h[i] = float(i % 97) * 0.01f;
  float* data; float* partial; uint32_t* count; uint32_t* dprog; float* dout;
  CK(hipMalloc(&data, n * sizeof(float)));
  CK(hipMemcpy(data, h.data(), n * sizeof(float), hipMemcpyHostToDevice));
  CK(hipMalloc(&partial, 1024 * sizeof(float)));
  CK(hipMalloc(&count, sizeof(uint32_t)));
  CK(hipMalloc(&dprog, kProgWords * sizeof(uint32_t)));
  CK(hipMalloc(&dout, sizeof(float)));
  uint32_t* dprog2; uint32_t* ddoor;
  CK(hipMalloc(&dprog2, kProgWords * sizeof(uint32_t)));
  CK(hipMalloc(&ddoor, sizeof(uint32_t)));
  Mailbox* mb;
  CK(hipHostMalloc((void**)&mb, sizeof(Mailbox), hipHostMallocDefault));
  std::memset(mb, 0, sizeof(Mailbox));
  float* hout;
  CK(hipHostMalloc((void**)&hout, sizeof(float), hipHostMallocDefault));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int reps = 3000;
  for (int nb : {64, 256}) {
    // ---- launch path
    auto call_launch = [&](uint32_t k) {
      mb->prog[0] = k;
      (void)hipMemcpyAsync(dprog, mb->prog, kProgWords * sizeof(uint32_t), hipMemcpyHostToDevice, s);
      k_work<<<nb, 256, 0, s>>>(dprog, data, n, partial);
      k_reduce<<<1, 64, 0, s>>>(partial, nb, dout);
      (void)hipMemcpyAsync(hout, dout, sizeof(float), hipMemcpyDeviceToHost, s);
      (void)hipStreamSynchronize(s);
      return *hout;
    };
    for (int i = 0; i < 200; ++i) call_launch(uint32_t(i));
    auto t0 = std::chrono::steady_clock::now();
    float acc = 0.0f;
    for (int i = 0; i < reps; ++i) acc += call_launch(uint32_t(i));
    const double us_launch = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count() / reps;
    const float ref = call_launch(77u);
    for (int variant = 1; variant <= 2; ++variant) {
    // ---- persistent path
    CK(hipMemsetAsync(count, 0, sizeof(uint32_t), s));
    CK(hipMemsetAsync(ddoor, 0, sizeof(uint32_t), s));
    CK(hipStreamSynchronize(s));
    mb->doorbell = 0; mb->done = 0; mb->stop = 0;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    const int max_idle = 200000;  // ~ tens of ms of idle polling, then the grid drains by itself
    if (variant == 1) k_persist<<<nb, 256, 0, s>>>(mb, data, n, partial, count, max_idle);
    else k_persist2<<<nb, 256, 0, s>>>(mb, data, n, partial, count, dprog2, ddoor, max_idle);
    CK(hipGetLastError());
    volatile Mailbox* vm = mb;
    bool ok = true;
    uint32_t seq = 0;
    auto call_persist = [&](uint32_t k) -> bool {
      vm->prog[0] = k;
      ++seq;
      std::atomic_thread_fence(std::memory_order_seq_cst);
      vm->doorbell = seq;
      auto ts = std::chrono::steady_clock::now();
      while (vm->done != seq) {
        if (std::chrono::steady_clock::now() - ts > std::chrono::milliseconds(200)) return false;
      }
      std::atomic_thread_fence(std::memory_order_seq_cst);
      return true;
    };
    for (int i = 0; i < 200 && ok; ++i) ok = call_persist(uint32_t(i));
    double us_persist = -1.0;
    float got = 0.0f;
    if (ok) {
      auto t1 = std::chrono::steady_clock::now();
      for (int i = 0; i < reps && ok; ++i) ok = call_persist(uint32_t(i));
      us_persist = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t1).count() / reps;
      if (ok) ok = call_persist(77u);
      got = vm->result;
    }
    vm->stop = 1;
    std::atomic_thread_fence(std::memory_order_seq_cst);
    CK(hipStreamSynchronize(s));  // the grid has drained
    std::printf("workgroups %4d: launch path %7.2f us per call, persistent v%d %7.2f us per call (%s); result %g vs %g %s\n",
                nb, us_launch, variant, us_persist, ok ? "ok" : "TIMED OUT", double(got), double(ref),
                ok && got == ref ? "equal" : "DIFFERENT");
    std::fflush(stdout);
    if (!ok) break;
    }
    (void)acc;
  }
  std::printf("done\n");
  return 0;
}
