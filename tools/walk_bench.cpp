// Micro-benchmark of the in-order fold's walk kernel (csrc/sr_aux.hip sr_fold_walk_kernel) on synthetic
// slow segments: np trees x n rows, every segment of rb_rows slow (its losses stored), losses uniform in
// [0.5, 1.5).  Prints the kernel time (HIP events) and the per-tree walk statistics.  Analysis only.
//   build: hipcc -O2 tools/walk_bench.cpp -Lsymbolicregression.jl_amd/lib -lsr_amd -o tools/walk_bench
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

struct SrFoldTabs {
  int32_t* code;
  void* tab;
  int32_t* sq;
  void* tab2;
};
struct SrFoldWho {  // (layout of csrc/sr_fold_dev.h's)
  const double* sums;
  const uint32_t* flags;
  int64_t n_terms;
  const uint8_t* elig;
  const double* est;
  int first;
  double* msum = nullptr;
  uint32_t* mflag = nullptr;
};
template <typename T>
hipError_t sr_launch_fold_walk(SrFoldTabs ft, const SrFoldWho& who, int np, int n_rb, int64_t rb_rows, int64_t n,
                               const T* losses, int64_t slot_rows, const uint32_t* perm, const T* carry, T* out_val,
                               int32_t* out_st, void* dbg, int all_rows, hipStream_t s);

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));       \
      return 1;                                                           \
    }                                                                     \
  } while (0)

int main(int argc, char** argv) {
  const int np = argc > 1 ? std::atoi(argv[1]) : 1;
  const int64_t n = argc > 2 ? std::atoll(argv[2]) : (1 << 20);
  const int64_t rb_rows = argc > 3 ? std::atoll(argv[3]) : 2048;
  const int every = argc > 4 ? std::atoi(argv[4]) : 1;  // every k-th segment slow (others: steps, not set up: fail)
  const int n_rb = int((n + rb_rows - 1) / rb_rows);
  std::vector<int32_t> code(size_t(n_rb) * np);
  for (int rb = 0; rb < n_rb; ++rb)
    for (int p = 0; p < np; ++p) code[size_t(rb) * np + p] = 0x40000000 + p * n_rb + rb;
  (void)every;
  std::vector<float> loss(size_t(np) * n_rb * rb_rows);
  std::mt19937 g(1);
  std::uniform_real_distribution<float> u(0.5f, 1.5f);
  for (auto& v : loss) v = u(g);
  int32_t *d_code, *d_st;
  float *d_loss, *d_val;
  int4* d_dbg;
  void* d_tab;
  CK(hipMalloc(&d_code, code.size() * 4));
  CK(hipMalloc(&d_loss, loss.size() * 4));
  CK(hipMalloc(&d_val, np * 4));
  CK(hipMalloc(&d_st, np * 4));
  CK(hipMalloc(&d_dbg, np * 16));
  CK(hipMalloc(&d_tab, code.size() * 8));
  CK(hipMemcpy(d_code, code.data(), code.size() * 4, hipMemcpyHostToDevice));
  int32_t* d_sq;
  CK(hipMalloc(&d_sq, code.size() * 4));
  CK(hipMemset(d_sq, 0x80, code.size() * 4));  // (0x80808080: a binade no running value has: rows)
  const SrFoldTabs ft{d_code, d_tab, d_sq, d_tab};
  CK(hipMemcpy(d_loss, loss.data(), loss.size() * 4, hipMemcpyHostToDevice));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 3; ++rep) {
    CK(hipEventRecord(e0, 0));
    CK(sr_launch_fold_walk<float>(ft, SrFoldWho{nullptr, nullptr, n, nullptr, nullptr, 1}, np, n_rb, rb_rows, n, d_loss, rb_rows, nullptr, nullptr, d_val, d_st, d_dbg, 1, 0));
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<int4> dbg(np);
    std::vector<int32_t> st(np);
    std::vector<float> val(np);
    CK(hipMemcpy(dbg.data(), d_dbg, np * 16, hipMemcpyDeviceToHost));
    CK(hipMemcpy(st.data(), d_st, np * 4, hipMemcpyDeviceToHost));
    CK(hipMemcpy(val.data(), d_val, np * 4, hipMemcpyDeviceToHost));
    // the host fold of tree 0
    float f = loss[0];
    for (int64_t i = 1; i < n; ++i) f = f + loss[size_t(i / rb_rows) * rb_rows + size_t(i % rb_rows)];
    std::printf("np %d n %lld rb_rows %lld: kernel %.3f ms; tree0 slow %d rounds %d slow-us %d walk-us %d st %d "
                "val %.9g host %.9g %s; per round %.3f us\n",
                np, (long long)n, (long long)rb_rows, ms, dbg[0].x, dbg[0].y, dbg[0].z, dbg[0].w, st[0], val[0], f,
                val[0] == f ? "EXACT" : "DIFF", dbg[0].y ? double(dbg[0].w) / dbg[0].y : 0.0);
  }
  return 0;
}
