// sr_grad_impl.h — batched forward-mode gradient of the loss with respect to tree constants.
//
// What it replaces: the objective/gradient pair BFGS calls in SymbolicRegression's constant
// optimisation (reference src/ConstantOptimization.jl:77-167: Evaluator / GradEvaluator with a
// forward-mode autodiff backend, i.e. value_and_gradient of eval_loss with respect to
// get_scalar_constants(tree)), for many (tree, constant vector) pairs in one launch.
//
// Execution model:
//   * a workgroup = W wave64s = W work items (tree, first tangent k0) x one row block; per tile the
//     X rows (all features), y and w are staged once in LDS and shared by the W waves;
//   * one row per lane; every value carries KT tangents (dual numbers with KT partials, the
//     constants k0 .. k0+KT-1 of the tree in pre-order), all in VGPRs; operand-stack slots
//     (value + tangents) live in a per-wave LDS area;
//   * constants come from a per-tree array (lane k holds constant k), so BFGS updates them without
//     recompiling; a constant leaf with slot c seeds the one-hot tangent e_{c-k0};
//   * per row, d loss / d pred (2(ŷ - y) for L2, sign for L1, times the weight) scales the tangents
//     into per-lane accumulators that live across the row block; one DPP wave reduction per
//     (item, tangent) at the end of the block -> [row block][item][KT] f64 partials.
// Only complete trees are differentiated (the caller evaluates the loss and `complete` with the
// exact loss kernel first: for an incomplete tree eval_loss is the constant L(Inf) and its
// gradient is zero), so this kernel needs no validity checks.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "sr_eval.h"
#include "sr_ops.h"
#include "sr_tile_impl.h"

// Value of lane l of v (l uniform).
template <typename T>
__device__ __forceinline__ T sr_readlane_val(T v, uint32_t l) {
  if constexpr (sizeof(T) == 4) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), int(l)));
  } else {
    const uint64_t b = uint64_t(__double_as_longlong(v));
    const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(b)), int(l)));
    const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(uint32_t(b >> 32)), int(l)));
    return __longlong_as_double(int64_t((uint64_t(hi) << 32) | lo));
  }
}

// Rows per lane by tangent width (8 for 1-2 tangents, 4 for 4, 2 for 8, 1 for 16): the value and its
// KT tangents of R rows stay in VGPRs, so one
// dispatch of an instruction covers R x 64 rows (round 3: one row per lane made every dispatch and
// operand decode cover 64 rows only; C3's gradient launches 0.61 ms each).
template <typename T, int KT>
struct SrGradRows {
  static constexpr int value = sr_grad_rows_per_lane(KT, int(sizeof(T)));
};

// R: rows per lane (SrGradRows' default, or 1 when the default's LDS operand stack would not fit:
// sr_grad_launch_rows)
template <typename T, int KT, int W, bool GATHER, int R>
__global__ void __launch_bounds__(W * 64) sr_grad_kernel(const SrGradArgs<T> a) {
  // rows per lane: lane + 64 j, j < R
  constexpr int ROWS = 64 * R;               // rows per staged tile
  constexpr int NV = 1 + KT;                 // value + tangents
  extern __shared__ __attribute__((aligned(16))) unsigned char sr_smem[];
  const int tid = threadIdx.x;
  const int wave = tid >> 6;
  const int lane = tid & 63;
  T* xs = reinterpret_cast<T*>(sr_smem);                       // [nf][ROWS]
  T* ys = xs + size_t(a.nf) * ROWS;                            // [ROWS]
  T* wsv = ys + ROWS;                                          // [ROWS] (weighted)
  T* stk = wsv + (a.w ? ROWS : 0);                             // [W][depth][NV][R][64]
  T* my_stk = stk + size_t(wave) * a.stack_depth * NV * R * 64 + lane;

  int tg, rb, item, item_end = a.n_items;
  const int64_t* ridx = a.row_idx;  // GATHER: this block's row view
  if (a.segs == nullptr) {
    tg = int(blockIdx.x) % a.n_groups;
    rb = int(blockIdx.x) / a.n_groups;
    item = tg * W + wave;
  } else {
    // several row views in one launch (sr_eval_grad_batch_views): segment = one view's work items
    int lo = 0, hi = a.n_segs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (a.segs[mid].block0 <= int(blockIdx.x)) lo = mid;
      else hi = mid - 1;
    }
    const SrSegment sg = a.segs[lo];
    const int local = int(blockIdx.x) - sg.block0;
    tg = local % sg.groups;
    rb = local / sg.groups;
    item = sg.pos0 + tg * W + wave;
    item_end = sg.pos0 + sg.n_pos;
    ridx += sg.row_off;
  }
  const bool active = item < item_end;
  uint32_t pb = 0u, pe = 0u, k0 = 0u, cb = 0u, nconst = 0u;
  if (active) {
    const uint32_t t = a.item_tree[item];
    pb = a.offsets[t];
    pe = a.offsets[t + 1];
    k0 = a.item_k0[item];
    cb = a.const_off[t];
    nconst = a.const_off[t + 1] - cb;
  }
  // this tree's constants: lane c holds constant c (programs are short: <= 64 constants per window
  // of lanes, more live in further registers of the same lane set)
  T cval0 = T(0), cval1 = T(0);
  if (active && uint32_t(lane) < nconst) cval0 = a.consts[cb + lane];
  if (active && uint32_t(lane) + 64u < nconst) cval1 = a.consts[cb + 64 + lane];

  double acc[KT];  // per-lane f64 accumulators across the row block
#pragma unroll
  for (int k = 0; k < KT; ++k) acc[k] = 0.0;
  const bool weighted = a.w != nullptr;
  sr_libm_lds_fill(tid, W * 64);  // libm tables (visible after the first tile's barrier)

  for (int tile = 0; tile < a.tiles_per_block; ++tile) {
    const int64_t row0 = (int64_t(rb) * a.tiles_per_block + tile) * ROWS;
    if (row0 >= a.n_rows) break;
    __syncthreads();
    for (int i = tid; i < ROWS; i += W * 64) {
      const int64_t v = row0 + i;
      const int64_t src = GATHER ? ridx[v < a.n_rows ? v : 0] : (v < a.n_rows ? v : 0);
      for (int f = 0; f < a.nf; ++f) xs[f * ROWS + i] = a.X[int64_t(f) * a.ld + src];
      ys[i] = a.y[src];
      if (weighted) wsv[i] = a.w[src];
    }
    __syncthreads();
    if (!active || pe == pb) continue;

    T v[R];
    T dv[R][KT];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      v[j] = T(0);
#pragma unroll
      for (int q = 0; q < KT; ++q) dv[j][q] = T(0);
    }
    for (uint32_t base = pb; base < pe; base += 64u) {
      uint4 cw = make_uint4(0u, 0u, 0u, 0u);
      if (base + lane < pe) cw = sr_load_window(a.code, base + lane);
      const uint32_t n_here = __builtin_amdgcn_readfirstlane((pe - base < 64u) ? pe - base : 64u);
      for (uint32_t k = 0; k < n_here; ++k) {
        const uint32_t opc = uint32_t(__builtin_amdgcn_readlane(int(cw.x), int(k)));
        const uint32_t meta = uint32_t(__builtin_amdgcn_readlane(int(cw.y), int(k)));
        const uint32_t idx = meta & SR_M_INDEX;  // feature / stack slot / constant slot
        uint32_t variant = 6u;
        if (opc >= SR_OP_BINARY0) variant = (opc - SR_OP_BINARY0) % 6u;
        const bool load = opc <= SR_OP_LOAD_CONST_PUSH;
        const bool from_feat = (load && (opc == SR_OP_LOAD_FEAT || opc == SR_OP_LOAD_FEAT_PUSH)) ||
                               variant == SR_V_FL || variant == SR_V_FR;
        const bool from_stack = variant == SR_V_SL || variant == SR_V_SR;
        // a constant operand: its value (wave-uniform) and its one-hot tangent e_{idx-k0}
        T cv = T(0);
        const int jj = int(idx) - int(k0);
        if (!from_feat && !from_stack)
          cv = idx < 64u ? sr_readlane_val<T>(cval0, idx) : sr_readlane_val<T>(cval1, idx - 64u);
        const T* xrow = xs + size_t(idx) * ROWS + lane;
        const T* sp = my_stk + size_t(idx) * NV * R * 64;
        if (load) {
          if (opc >= SR_OP_LOAD_FEAT_PUSH) {
            T* pp = my_stk + size_t(((meta >> SR_M_PUSH_SHIFT) & 0x3fu) - 1u) * NV * R * 64;
#pragma unroll
            for (int j = 0; j < R; ++j) {
              pp[j * 64] = v[j];
#pragma unroll
              for (int q = 0; q < KT; ++q) pp[((q + 1) * R + j) * 64] = dv[j][q];
            }
          }
#pragma unroll
          for (int j = 0; j < R; ++j) {
            v[j] = from_feat ? xrow[j * 64] : cv;
#pragma unroll
            for (int q = 0; q < KT; ++q) dv[j][q] = (!from_feat && q == jj) ? T(1) : T(0);
          }
        } else if (opc < SR_OP_BINARY0) {
          const uint32_t u = opc >= SR_OP_UNARY_INF0 ? opc - SR_OP_UNARY_INF0 : opc - SR_OP_UNARY0;
          // the operator chosen once per instruction (a compile-time operator inside the row loop),
          // not once per row; operators outside the BASIC set take the generic loop
          auto unary_rows = [&](auto op_c) {
            constexpr uint32_t UID = decltype(op_c)::value;
            const uint32_t uu = UID == 0xffffffffu ? u : UID;
#pragma unroll
            for (int j = 0; j < R; ++j) {
              const T x = v[j];
              const T yv = sr_unary<T>(uu, x);
              // (fused unaries: complete trees have finite inner values, so INFSUB never fires)
              const T dfx = sr_unary_deriv<T>(uu, x, yv);
              v[j] = yv;
#pragma unroll
              for (int q = 0; q < KT; ++q) dv[j][q] = dfx * dv[j][q];
            }
          };
#define SR_GU(ID) \
  case ID: unary_rows(std::integral_constant<uint32_t, ID>{}); break;
          switch (u) {
            SR_GU(SR_U_NEG) SR_GU(SR_U_SQUARE) SR_GU(SR_U_CUBE) SR_GU(SR_U_EXP) SR_GU(SR_U_COS)
            SR_GU(SR_U_SIN) SR_GU(SR_U_LOG) SR_GU(SR_U_SQRT) SR_GU(SR_U_ABS)
            default: unary_rows(std::integral_constant<uint32_t, 0xffffffffu>{}); break;
          }
#undef SR_GU
        } else {
          const uint32_t b = (opc - SR_OP_BINARY0) / 6u + 1u;
          const bool left = variant == SR_V_SL || variant == SR_V_FL || variant == SR_V_CL;
          auto binary_rows = [&](auto op_c) {
            constexpr uint32_t BID = decltype(op_c)::value;
            const uint32_t bb = BID == 0xffffffffu ? b : BID;
#pragma unroll
            for (int j = 0; j < R; ++j) {
              // operand (value + tangents) of row j: feature / stack slot / constant
              T ov, od[KT];
              if (from_feat) {
                ov = xrow[j * 64];
#pragma unroll
                for (int q = 0; q < KT; ++q) od[q] = T(0);
              } else if (from_stack) {
                ov = sp[j * 64];
#pragma unroll
                for (int q = 0; q < KT; ++q) od[q] = sp[((q + 1) * R + j) * 64];
              } else {
                ov = cv;
#pragma unroll
                for (int q = 0; q < KT; ++q) od[q] = q == jj ? T(1) : T(0);
              }
              const T av = left ? ov : v[j], bv = left ? v[j] : ov;
              const T rv = sr_binary<T>(bb, av, bv);
              T pa, pbv;
              sr_binary_partials<T>(bb, av, bv, rv, &pa, &pbv);
              v[j] = rv;
              if (left) {
#pragma unroll
                for (int q = 0; q < KT; ++q) dv[j][q] = __builtin_fma(pa, od[q], pbv * dv[j][q]);
              } else {
#pragma unroll
                for (int q = 0; q < KT; ++q) dv[j][q] = __builtin_fma(pa, dv[j][q], pbv * od[q]);
              }
            }
          };
          switch (b) {
            case SR_B_ADD: binary_rows(std::integral_constant<uint32_t, SR_B_ADD>{}); break;
            case SR_B_SUB: binary_rows(std::integral_constant<uint32_t, SR_B_SUB>{}); break;
            case SR_B_MUL: binary_rows(std::integral_constant<uint32_t, SR_B_MUL>{}); break;
            case SR_B_DIV: binary_rows(std::integral_constant<uint32_t, SR_B_DIV>{}); break;
            default: binary_rows(std::integral_constant<uint32_t, 0xffffffffu>{}); break;
          }
        }
      }
    }
    // d loss / d constant: (d loss / d pred) * d pred / d constant, padded rows excluded
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int r = j * 64 + lane;
      T coef = sr_elem_loss_deriv<T>(a.loss_kind, v[j], ys[r], a.loss_param);
      if (weighted) coef *= wsv[r];
      if (row0 + r >= a.n_rows) coef = T(0);
#pragma unroll
      for (int q = 0; q < KT; ++q) acc[q] = __builtin_fma(double(coef), double(dv[j][q]), acc[q]);
    }
  }
  if (!active) return;
#pragma unroll
  for (int q = 0; q < KT; ++q) {
    const double s = sr_wave_sum<double>(acc[q]);
    if (lane == 0) a.part[(size_t(rb) * a.n_items + item) * KT + q] = s;
  }
}

template <typename T, int KT, int W, bool GATHER, int R>
hipError_t sr_launch_grad(const SrGradArgs<T>& a, int n_blocks, hipStream_t s) {
  const size_t lds = sr_grad_lds_bytes(int(sizeof(T)), KT, R, a.nf, a.w != nullptr, a.stack_depth, W);
  const void* fn = reinterpret_cast<const void*>(&sr_grad_kernel<T, KT, W, GATHER, R>);
  if (lds > 65536) {
    const hipError_t e = hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, int(lds));
    if (e != hipSuccess) return e;
  }
  hipLaunchKernelGGL((sr_grad_kernel<T, KT, W, GATHER, R>), dim3(n_blocks), dim3(W * 64), lds, s, a);
  return hipGetLastError();
}

// Σ over row blocks of the [row block][item][KT] partials -> out[item][KT], one wave per value: lane
// l folds row blocks l, l + 64, ... in order and a fixed butterfly adds the lanes (deterministic; a
// thread per value walking ~160 row blocks serially took 46 us per launch in C3's searches).
__global__ void __launch_bounds__(256) sr_grad_reduce_kernel(const double* __restrict__ part, int n_row_blocks,
                                                              int n_vals, double* __restrict__ out) {
  const int lane = int(threadIdx.x) & 63;
  const int i = int(int64_t(blockIdx.x) * (blockDim.x / 64) + threadIdx.x / 64);
  if (i >= n_vals) return;  // wave-uniform
  double s = 0.0;
  for (int b = lane; b < n_row_blocks; b += 64) s += part[size_t(b) * n_vals + i];
#pragma unroll
  for (int off = 32; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
  if (lane == 0) out[i] = s;
}
