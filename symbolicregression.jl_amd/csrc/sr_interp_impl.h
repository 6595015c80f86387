// sr_eval.hip — CDNA4 (gfx950) batched expression-tree interpreter.
//
// What it replaces: DynamicExpressions' array-at-a-time `eval_tree_array` + SymbolicRegression's
// `_eval_loss` (reference src/LossFunctions.jl:90-117), for a whole population at once.
//
// Execution model:
//   * one workgroup = 4 wave64s = 256 lanes; each lane owns R consecutive rows (R*sizeof(T) = 16 B,
//     one coalesced dwordx4 load per feature); a workgroup owns `tiles` row tiles of 256*R rows and a
//     group of G trees;
//   * every wave interprets the SAME program word stream (scalar loads -> wave-uniform control flow);
//     one flat `switch` over an 8-bit combined opcode (operation + operand source) dispatches to
//     straight-line VALU bodies that update the R-row top of stack in place;
//   * the top of stack lives in VGPRs, deeper slots in a per-wave LDS stack (Sethi–Ullman ordering
//     keeps it <= 3 deep for maxsize 30); the X tile stays in VGPRs for all G trees (a feature index
//     becomes one `s_set_gpr_idx_on` indexed read); y / weights of the tile wait in LDS;
//   * DynamicExpressions' early-exit checks become ballots: a CHECK instruction tests |v| < tbig; a
//     non-finite value ends the tree for the wave (and, via LDS, for the whole workgroup);
//   * per-tree loss: T per lane -> cross-lane wave sum -> f64 accumulators in LDS -> one partial per
//     (tree, row block) -> fixed-order reduce kernel (bit-reproducible).
// The kernel must be compiled with -mllvm -structurizecfg-skip-uniform-regions=true: all its branches
// are wave-uniform, and without the flag LLVM's structurizer turns the opcode switch into a chain of
// exec-mask "flow" blocks with copies of the stack registers at every join.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "sr_ops.h"
#include "sr_eval.h"

#define SR_WAVES 4
#define SR_BLOCK (SR_WAVES * 64)
#define SR_STACK_DEPTH 4

// R values per lane moved as 16-byte vectors (dwordx4 / ds_*_b128).
template <typename T>
struct SrChunk;
template <>
struct SrChunk<float> {
  using V = float4;
  static constexpr int N = 4;
  static __device__ inline void get(const V& v, float* o) { o[0] = v.x; o[1] = v.y; o[2] = v.z; o[3] = v.w; }
  static __device__ inline V make(const float* o) { return make_float4(o[0], o[1], o[2], o[3]); }
};
template <>
struct SrChunk<double> {
  using V = double2;
  static constexpr int N = 2;
  static __device__ inline void get(const V& v, double* o) { o[0] = v.x; o[1] = v.y; }
  static __device__ inline V make(const double* o) { return make_double2(o[0], o[1]); }
};
template <typename T, int R>
struct SrVec {
  using C = SrChunk<T>;
  static_assert(R % C::N == 0, "rows per lane must fill whole 16-byte vectors");
  static __device__ inline void load(const T* p, T (&o)[R]) {
#pragma unroll
    for (int c = 0; c < R / C::N; ++c) C::get(reinterpret_cast<const typename C::V*>(p)[c], o + c * C::N);
  }
  static __device__ inline void store(T* p, const T (&o)[R]) {
#pragma unroll
    for (int c = 0; c < R / C::N; ++c) reinterpret_cast<typename C::V*>(p)[c] = C::make(o + c * C::N);
  }
};

template <typename T>
__device__ __forceinline__ T sr_wave_sum(T v) {
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}
__device__ __forceinline__ uint64_t sr_ballot(bool p) { return __builtin_amdgcn_ballot_w64(p); }

// Feature operand X[f] for this lane's R rows.  Small tiles use one indexed register read
// (s_set_gpr_idx_on + R moves); tiles above 32 registers would be demoted to scratch by LLVM when
// indexed dynamically, so they branch on the (wave-uniform) feature index instead.
template <typename T, int R, int FCAP>
__device__ __forceinline__ void sr_fetch_feature(const T (&xr)[FCAP][R], uint32_t f, T (&o)[R]) {
  if constexpr (FCAP * R <= 32) {
#pragma unroll
    for (int r = 0; r < R; ++r) o[r] = xr[f][r];
  } else {
#define SR_FCASE(K)                                        \
  case K:                                                  \
    if constexpr (K < FCAP) {                              \
      _Pragma("unroll") for (int r = 0; r < R; ++r) o[r] = xr[K][r]; \
    }                                                      \
    break;
    switch (f) {
      SR_FCASE(0) SR_FCASE(1) SR_FCASE(2) SR_FCASE(3) SR_FCASE(4) SR_FCASE(5) SR_FCASE(6) SR_FCASE(7)
      SR_FCASE(8) SR_FCASE(9) SR_FCASE(10) SR_FCASE(11) SR_FCASE(12) SR_FCASE(13) SR_FCASE(14) SR_FCASE(15)
      default:
        break;
    }
#undef SR_FCASE
  }
}

// ------------------------------------------------------------------ dispatch cases
// Operators of the BASIC tier are compiled into every kernel; the FULL tier adds the rest of the
// catalog (more registers: transcendental constants are hoisted out of the loop by LLVM).
#define SR_EACH(EXPR)                                     \
  _Pragma("unroll") for (int r = 0; r < R; ++r) {         \
    const T x = tos[r];                                   \
    tos[r] = (EXPR);                                      \
  }
#define SR_UCASE(ID)                                      \
  case SR_OP_UNARY0 + ID: {                               \
    SR_EACH(sr_unary<T>(ID, x));                          \
    break;                                                \
  }
#define SR_UCASE_FULL(ID)                                 \
  case SR_OP_UNARY0 + ID: {                               \
    if (TIER == SR_TIER_FULL) {                           \
      SR_EACH(sr_unary<T>(ID, x));                        \
    }                                                     \
    break;                                                \
  }
#define SR_BIN_EACH(AEXPR, BEXPR, ID)                     \
  _Pragma("unroll") for (int r = 0; r < R; ++r) {         \
    const T aa = (AEXPR);                                 \
    const T bb = (BEXPR);                                 \
    tos[r] = sr_binary<T>(ID, aa, bb);                    \
  }
#define SR_BCASE_GEN(ID, ENABLED)                                                              \
  case SR_BIN_OPC(ID, SR_V_SL): {                                                              \
    if (ENABLED) {                                                                             \
      --sp;                                                                                    \
      T o[R];                                                                                  \
      SrVec<T, R>::load(stk + size_t(sp) * 64 * R, o);                                         \
      SR_BIN_EACH(o[r], tos[r], ID);                                                           \
    }                                                                                          \
    break;                                                                                     \
  }                                                                                            \
  case SR_BIN_OPC(ID, SR_V_SR): {                                                              \
    if (ENABLED) {                                                                             \
      --sp;                                                                                    \
      T o[R];                                                                                  \
      SrVec<T, R>::load(stk + size_t(sp) * 64 * R, o);                                         \
      SR_BIN_EACH(tos[r], o[r], ID);                                                           \
    }                                                                                          \
    break;                                                                                     \
  }                                                                                            \
  case SR_BIN_OPC(ID, SR_V_FL): {                                                              \
    if (ENABLED) {                                                                             \
      T o[R];                                                                                  \
      sr_fetch_feature<T, R, FCAP>(xr, in.arg, o);                                             \
      SR_BIN_EACH(o[r], tos[r], ID);                                                           \
    }                                                                                          \
    break;                                                                                     \
  }                                                                                            \
  case SR_BIN_OPC(ID, SR_V_FR): {                                                              \
    if (ENABLED) {                                                                             \
      T o[R];                                                                                  \
      sr_fetch_feature<T, R, FCAP>(xr, in.arg, o);                                             \
      SR_BIN_EACH(tos[r], o[r], ID);                                                           \
    }                                                                                          \
    break;                                                                                     \
  }                                                                                            \
  case SR_BIN_OPC(ID, SR_V_CL): {                                                              \
    if (ENABLED) {                                                                             \
      const T cv = in.val;                                                                     \
      SR_BIN_EACH(cv, tos[r], ID);                                                             \
    }                                                                                          \
    break;                                                                                     \
  }                                                                                            \
  case SR_BIN_OPC(ID, SR_V_CR): {                                                              \
    if (ENABLED) {                                                                             \
      const T cv = in.val;                                                                     \
      SR_BIN_EACH(tos[r], cv, ID);                                                             \
    }                                                                                          \
    break;                                                                                     \
  }
#define SR_BCASE(ID) SR_BCASE_GEN(ID, true)
#define SR_BCASE_FULL(ID) SR_BCASE_GEN(ID, TIER == SR_TIER_FULL)

// ------------------------------------------------------------------ the interpreter kernel
// MODE: SR_MODE_LOSS (partials), SR_MODE_PRED (write predictions), SR_MODE_EXACT (check sums).
// VAR bit 0: prefetch the next program word while the current one executes.
template <typename T, int R, int FCAP, int MODE, bool GATHER, int TIER, int VAR>
__global__ void __launch_bounds__(SR_BLOCK) sr_interp_kernel(const SrEvalArgs<T> a) {
  constexpr int D = SR_STACK_DEPTH;
  extern __shared__ __attribute__((aligned(16))) unsigned char sr_smem[];
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  const int G = a.trees_per_block;

  // LDS carve (all 16-byte aligned):
  //   stack [SR_WAVES][D][64][R] T | acc [SR_WAVES][G] f64 | flg [SR_WAVES][G] u32 | abort [G] u32
  T* stk = reinterpret_cast<T*>(sr_smem) + (size_t(wave) * D * 64 + lane) * R;
  double* acc = reinterpret_cast<double*>(reinterpret_cast<T*>(sr_smem) + size_t(SR_WAVES) * D * 64 * R);
  uint32_t* flg = reinterpret_cast<uint32_t*>(acc + SR_WAVES * G);
  uint32_t* abort_flag = flg + SR_WAVES * G;
  // EXACT mode: per-wave check-sum accumulators [SR_WAVES][max_checks] after the abort words
  double* xacc = reinterpret_cast<double*>(abort_flag + ((G + 3) & ~3));
  const int MC = (MODE == SR_MODE_EXACT) ? a.max_checks : 0;

  const int rb = blockIdx.x % a.n_row_blocks;
  const int tg = blockIdx.x / a.n_row_blocks;

  for (int i = tid; i < SR_WAVES * G; i += SR_BLOCK) {
    acc[i] = 0.0;
    flg[i] = 0u;
  }
  for (int i = tid; i < G; i += SR_BLOCK) abort_flag[i] = 0u;
  for (int i = tid; i < SR_WAVES * MC; i += SR_BLOCK) xacc[i] = 0.0;
  __syncthreads();

  const int tree0 = tg * G;
  int gcount = a.n_trees - tree0;
  if (gcount > G) gcount = G;
  const bool weighted = a.w != nullptr;

  for (int tile = 0; tile < a.tiles_per_block; ++tile) {
    const int64_t row0 = ((int64_t(rb) * a.tiles_per_block + tile) * SR_BLOCK + tid) * R;
    if (!sr_ballot(row0 < a.n_rows)) continue;  // whole wave past the end (uniform)

    // ---- stage this lane's R rows of X in VGPRs (y / w are re-read at each tree's loss: L1/L2 hits)
    T xr[FCAP][R];
    bool valid[R];
#pragma unroll
    for (int r = 0; r < R; ++r) valid[r] = (row0 + r) < a.n_rows;
    int64_t idx[R];
    if (GATHER) {
#pragma unroll
      for (int r = 0; r < R; ++r) idx[r] = a.row_idx[valid[r] ? row0 + r : 0];  // pad with row 0 of the view
#pragma unroll
      for (int f = 0; f < FCAP; ++f) {
#pragma unroll
        for (int r = 0; r < R; ++r) xr[f][r] = (f < a.nf) ? a.X[int64_t(f) * a.ld + idx[r]] : T(0);
      }
    } else {
#pragma unroll
      for (int f = 0; f < FCAP; ++f) {
        if (f < a.nf) {
          SrVec<T, R>::load(a.X + int64_t(f) * a.ld + row0, xr[f]);
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) xr[f][r] = T(0);
        }
      }
    }

    for (int g = 0; g < gcount; ++g) {
      const int tree = (MODE == SR_MODE_EXACT) ? int(a.tree_list[tree0 + g]) : tree0 + g;
      if (MODE == SR_MODE_LOSS && __builtin_amdgcn_readfirstlane(abort_flag[g])) continue;
      const uint32_t pb = a.offsets[tree];
      const uint32_t pe = a.offsets[tree + 1];
      if (pb == pe) continue;  // statically incomplete (constant checks)

      T tos[R];
#pragma unroll
      for (int r = 0; r < R; ++r) tos[r] = T(0);
      int sp = 0;
      bool dead = false;
      int check_k = 0;
      uint64_t susp_any = 0;

      SrIns<T> nxt = a.code[pb];
      for (uint32_t pc = pb; pc < pe; ++pc) {
        SrIns<T> in;
        if (VAR & 1) {
          in = nxt;
          nxt = a.code[pc + 1];  // the program buffer is padded by one instruction
        } else {
          in = a.code[pc];
        }
        const uint32_t c = in.code;
        T save[R];
        if (c & SR_F_INFSUB) {
#pragma unroll
          for (int r = 0; r < R; ++r) save[r] = tos[r];
        }
        switch (SR_OPC(c)) {
          case SR_OP_LOAD_FEAT: {
            sr_fetch_feature<T, R, FCAP>(xr, in.arg, tos);
            break;
          }
          case SR_OP_LOAD_CONST: {
#pragma unroll
            for (int r = 0; r < R; ++r) tos[r] = in.val;
            break;
          }
          case SR_OP_LOAD_FEAT_PUSH: {
            SrVec<T, R>::store(stk + size_t(sp) * 64 * R, tos);
            ++sp;
            sr_fetch_feature<T, R, FCAP>(xr, in.arg, tos);
            break;
          }
          case SR_OP_LOAD_CONST_PUSH: {
            SrVec<T, R>::store(stk + size_t(sp) * 64 * R, tos);
            ++sp;
#pragma unroll
            for (int r = 0; r < R; ++r) tos[r] = in.val;
            break;
          }
          // BASIC tier
          SR_UCASE(SR_U_NEG) SR_UCASE(SR_U_SQUARE) SR_UCASE(SR_U_CUBE) SR_UCASE(SR_U_EXP)
          SR_UCASE(SR_U_COS) SR_UCASE(SR_U_SIN) SR_UCASE(SR_U_LOG) SR_UCASE(SR_U_SQRT)
          SR_UCASE(SR_U_ABS)
          SR_BCASE(SR_B_ADD) SR_BCASE(SR_B_SUB) SR_BCASE(SR_B_MUL) SR_BCASE(SR_B_DIV)
          // FULL tier
          SR_UCASE_FULL(SR_U_TAN) SR_UCASE_FULL(SR_U_LOG2) SR_UCASE_FULL(SR_U_LOG10)
          SR_UCASE_FULL(SR_U_LOG1P) SR_UCASE_FULL(SR_U_SIGN) SR_UCASE_FULL(SR_U_TANH)
          SR_UCASE_FULL(SR_U_SINH) SR_UCASE_FULL(SR_U_COSH) SR_UCASE_FULL(SR_U_ATAN)
          SR_UCASE_FULL(SR_U_ASIN) SR_UCASE_FULL(SR_U_ACOS) SR_UCASE_FULL(SR_U_ACOSH)
          SR_UCASE_FULL(SR_U_ATANH) SR_UCASE_FULL(SR_U_ASINH) SR_UCASE_FULL(SR_U_RELU)
          SR_UCASE_FULL(SR_U_INV) SR_UCASE_FULL(SR_U_ERF) SR_UCASE_FULL(SR_U_ERFC)
          SR_UCASE_FULL(SR_U_GAMMA) SR_UCASE_FULL(SR_U_ROUND) SR_UCASE_FULL(SR_U_FLOOR)
          SR_UCASE_FULL(SR_U_CEIL) SR_UCASE_FULL(SR_U_EXP2) SR_UCASE_FULL(SR_U_EXPM1)
          SR_BCASE_FULL(SR_B_POW) SR_BCASE_FULL(SR_B_MAX) SR_BCASE_FULL(SR_B_MIN)
          SR_BCASE_FULL(SR_B_MOD) SR_BCASE_FULL(SR_B_GREATER) SR_BCASE_FULL(SR_B_LESS)
          SR_BCASE_FULL(SR_B_GREATER_EQUAL) SR_BCASE_FULL(SR_B_LESS_EQUAL) SR_BCASE_FULL(SR_B_COND)
          SR_BCASE_FULL(SR_B_LOGICAL_OR) SR_BCASE_FULL(SR_B_LOGICAL_AND) SR_BCASE_FULL(SR_B_ATAN2)
          default:
            break;
        }
        if (c & (SR_F_INFSUB | SR_F_CHECK)) {
          if (c & SR_F_INFSUB) {
#pragma unroll
            for (int r = 0; r < R; ++r) tos[r] = sr_isfinite(save[r]) ? tos[r] : sr_inf<T>();
          }
          if (c & SR_F_CHECK) {
            if (MODE == SR_MODE_EXACT) {
              double s = 0.0;
#pragma unroll
              for (int r = 0; r < R; ++r) s += valid[r] ? double(tos[r]) * a.scale : 0.0;
              s = sr_wave_sum<double>(s);
              if (lane == 0) xacc[wave * MC + check_k] += s;
              ++check_k;
            } else {
              // padded rows replicate row 0 of the view, so no row mask is needed here
              bool susp = false;
#pragma unroll
              for (int r = 0; r < R; ++r) susp |= !(SrM<T>::fabs(tos[r]) < a.tbig);
              const uint64_t sm = sr_ballot(susp);
              if (sm) {
                susp_any |= sm;
                bool nonfin = false;
#pragma unroll
                for (int r = 0; r < R; ++r) nonfin |= !sr_isfinite(tos[r]);
                if (sr_ballot(nonfin)) {
                  dead = true;
                  break;
                }
              }
            }
          }
        }
      }

      if (MODE == SR_MODE_LOSS) {
        if (dead) {
          if (lane == 0) {
            flg[wave * G + g] |= SR_FLAG_NONFINITE;
            abort_flag[g] = 1u;
          }
          continue;
        }
        T yv[R];
        if (GATHER) {
#pragma unroll
          for (int r = 0; r < R; ++r) yv[r] = a.y[idx[r]];
        } else {
          SrVec<T, R>::load(a.y + row0, yv);
        }
        T s = T(0);
        if (weighted) {
          T wv[R];
          if (GATHER) {
#pragma unroll
            for (int r = 0; r < R; ++r) wv[r] = a.w[idx[r]];
          } else {
            SrVec<T, R>::load(a.w + row0, wv);
          }
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const T l = sr_elem_loss<T>(a.loss_kind, tos[r], yv[r]) * wv[r];
            s += valid[r] ? l : T(0);
          }
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) {
            const T l = sr_elem_loss<T>(a.loss_kind, tos[r], yv[r]);
            s += valid[r] ? l : T(0);
          }
        }
        s = sr_wave_sum<T>(s);
        if (lane == 0) {
          acc[wave * G + g] += double(s);
          if (susp_any) flg[wave * G + g] |= SR_FLAG_BIG;
        }
      } else if (MODE == SR_MODE_PRED) {
        T* out = a.pred + int64_t(tree) * a.pred_ld;
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (valid[r]) out[row0 + r] = dead ? sr_qnan<T>() : tos[r];
        if (lane == 0) {
          if (dead) flg[wave * G + g] |= SR_FLAG_NONFINITE;
          else if (susp_any) flg[wave * G + g] |= SR_FLAG_BIG;
        }
      }
    }
  }

  __syncthreads();
  if (MODE == SR_MODE_EXACT) {
    // one device-scope add per (block, check): 256-way instead of 4096-way contention per word
    for (int k = tid; k < MC; k += SR_BLOCK) {
      double v = 0.0;
#pragma unroll
      for (int w = 0; w < SR_WAVES; ++w) v += xacc[w * MC + k];
      if (v != 0.0) atomicAdd(a.check_sums + size_t(tree0) * MC + k, v);
    }
    return;
  }
  for (int g = tid; g < gcount; g += SR_BLOCK) {
    double s = 0.0;
    uint32_t f = 0u;
#pragma unroll
    for (int w = 0; w < SR_WAVES; ++w) {
      s += acc[w * G + g];
      f |= flg[w * G + g];
    }
    const size_t o = size_t(tree0 + g) * a.n_row_blocks + rb;
    a.part_sum[o] = s;
    a.part_flag[o] = f;
  }
}

// ------------------------------------------------------------------ launch helpers
template <typename T>
size_t sr_interp_lds_bytes(int trees_per_block, int rows_per_lane, int max_checks) {
  return size_t(SR_WAVES) * SR_STACK_DEPTH * 64 * rows_per_lane * sizeof(T) +
         size_t(SR_WAVES) * trees_per_block * 8 + size_t(SR_WAVES) * trees_per_block * 4 +
         size_t((trees_per_block + 3) & ~3) * 4 + size_t(SR_WAVES) * max_checks * 8;
}

template <typename T, int R, int FCAP, int MODE, bool GATHER, int TIER, int VAR>
static hipError_t launch_interp(const SrEvalArgs<T>& a, int n_blocks, hipStream_t s) {
  const size_t lds = sr_interp_lds_bytes<T>(a.trees_per_block, R, MODE == SR_MODE_EXACT ? a.max_checks : 0);
  hipLaunchKernelGGL((sr_interp_kernel<T, R, FCAP, MODE, GATHER, TIER, VAR>), dim3(n_blocks), dim3(SR_BLOCK), lds, s,
                     a);
  return hipGetLastError();
}

template <typename T, int R, int MODE, bool GATHER, int TIER, int VAR>
hipError_t sr_dispatch_interp(const SrEvalArgs<T>& a, int n_blocks, hipStream_t s) {
  if (a.nf <= 4) return launch_interp<T, R, 4, MODE, GATHER, TIER, VAR>(a, n_blocks, s);
  if (a.nf <= 8) return launch_interp<T, R, 8, MODE, GATHER, TIER, VAR>(a, n_blocks, s);
  return launch_interp<T, R, SR_MAX_FEATURES, MODE, GATHER, TIER, VAR>(a, n_blocks, s);
}

// Explicit instantiations are spread over several translation units (sr_inst_*.hip, one per
// element type / mode) so the build compiles them in parallel; see the Makefile.
#define SR_INSTANTIATE(T, R, MODE, GATHER, TIER, VAR) \
  template hipError_t sr_dispatch_interp<T, R, MODE, GATHER, TIER, VAR>(const SrEvalArgs<T>&, int, hipStream_t);
