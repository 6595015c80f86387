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

// Row callees (noinline: their temporaries live in the callee's own registers, so the kernel's VGPR
// count — and with it its occupancy — is set by the interpreter loop, not by the largest operator body;
// round 3's Float64 kernels inlined every operator into a row-unrolled switch: 256 VGPRs, one wave per
// SIMD).  Value rows, derivative rows, and the operators outside the BASIC set.
template <typename T, int R>
using SrGVec = T __attribute__((ext_vector_type(R)));
template <typename T, int R>
__device__ __attribute__((noinline)) SrGVec<T, R> sr_grad_unary_val(uint32_t u, SrGVec<T, R> x) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    x[r] = sr_unary<T>(u, x[r]);
    __builtin_amdgcn_sched_barrier(0);
  }
  return x;
}
template <typename T, int R>
__device__ __attribute__((noinline)) SrGVec<T, R> sr_grad_unary_der(uint32_t u, SrGVec<T, R> x, SrGVec<T, R> y) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    x[r] = sr_unary_deriv<T>(u, x[r], y[r]);
    __builtin_amdgcn_sched_barrier(0);
  }
  return x;
}
template <typename T, int R>
__device__ __attribute__((noinline)) SrGVec<T, R> sr_grad_binary_val(uint32_t b, SrGVec<T, R> x, SrGVec<T, R> y) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    x[r] = sr_binary<T>(b, x[r], y[r]);
    __builtin_amdgcn_sched_barrier(0);
  }
  return x;
}
// WHICH = 0: d r / d a, 1: d r / d b
template <typename T, int R, int WHICH>
__device__ __attribute__((noinline)) SrGVec<T, R> sr_grad_binary_der(uint32_t b, SrGVec<T, R> x, SrGVec<T, R> y,
                                                                      SrGVec<T, R> res) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    T pa, pb;
    sr_binary_partials<T>(b, x[r], y[r], res[r], &pa, &pb);
    x[r] = WHICH == 0 ? pa : pb;
    __builtin_amdgcn_sched_barrier(0);
  }
  return x;
}
template <typename T, int R>
__device__ __attribute__((noinline)) SrGVec<T, R> sr_grad_loss_der(int kind, SrGVec<T, R> pred, SrGVec<T, R> y, T p) {
#pragma unroll
  for (int r = 0; r < R; ++r) {
    pred[r] = sr_elem_loss_deriv<T>(kind, pred[r], y[r], p);
    __builtin_amdgcn_sched_barrier(0);
  }
  return pred;
}

// R: rows per lane (sr_grad_launch_rows: up to 8 for 1-2 tangents, 4 for 4, 2 for 8, 1 for 16): the
// value and its KT tangents of R rows stay in VGPRs, so one dispatch of an instruction covers R x 64
// rows (round 3: one row per lane made every dispatch and operand decode cover 64 rows only).
template <typename T, int KT, int W, bool GATHER, int R>
__global__ void __launch_bounds__(W * 64) sr_grad_kernel(const SrGradArgs<T> a) {
  // rows per lane: lane + 64 j, j < R; a staged tile of TROWS rows is interpreted in TROWS / ROWS
  // sub-passes (round 5: one barrier pair and one staging round per 256 rows, not per 64 R; a lane
  // still meets its rows in row order, so the sums are the same bit for bit)
  constexpr int ROWS = 64 * R;                      // rows per program pass
  constexpr int TROWS = sr_grad_tile_rows(R);       // rows per staged tile
  constexpr int SUBS = TROWS / ROWS;
  static_assert(TROWS % ROWS == 0, "tile rows");
  constexpr int NV = 1 + KT;                 // value + tangents
  extern __shared__ __attribute__((aligned(16))) unsigned char sr_smem[];
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // (uniform: item, k0 and jj live in SGPRs)
  const int lane = tid & 63;
  T* xs = reinterpret_cast<T*>(sr_smem);                       // [nf][TROWS]
  T* ys = xs + size_t(a.nf) * TROWS;                           // [TROWS]
  T* wsv = ys + TROWS;                                         // [TROWS] (weighted)
  T* stk = wsv + (a.w ? TROWS : 0);                            // [W][depth][NV][R][64]
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
    const int64_t tile0 = (int64_t(rb) * a.tiles_per_block + tile) * TROWS;
    if (tile0 >= a.n_rows) break;
    __syncthreads();
    for (int i = tid; i < TROWS; i += W * 64) {
      const int64_t v = tile0 + i;
      const int64_t src = GATHER ? ridx[v < a.n_rows ? v : 0] : (v < a.n_rows ? v : 0);
      for (int f = 0; f < a.nf; ++f) xs[f * TROWS + i] = a.X[int64_t(f) * a.ld + src];
      ys[i] = a.y[src];
      if (weighted) wsv[i] = a.w[src];
    }
    __syncthreads();
    if (!active || pe == pb) continue;
    // the program's first window, kept across the sub-passes (programs are almost always <= 64)
    uint4 cw0 = make_uint4(0u, 0u, 0u, 0u);
    if (pb + lane < pe) cw0 = sr_load_window(a.code, pb + lane);
    for (int sub = 0; sub < SUBS; ++sub) {
    const int ro = sub * ROWS;  // the sub-pass's first row in the tile
    const int64_t row0 = tile0 + ro;
    if (row0 >= a.n_rows) break;

    T v[R];
    T dv[R][KT];
#pragma unroll
    for (int j = 0; j < R; ++j) {
      v[j] = T(0);
#pragma unroll
      for (int q = 0; q < KT; ++q) dv[j][q] = T(0);
    }
    for (uint32_t base = pb; base < pe; base += 64u) {
      uint4 cw = cw0;
      if (base != pb) {
        cw = make_uint4(0u, 0u, 0u, 0u);
        if (base + lane < pe) cw = sr_load_window(a.code, base + lane);
      }
      const uint32_t n_here = __builtin_amdgcn_readfirstlane((pe - base < 64u) ? pe - base : 64u);
      for (uint32_t k = 0; k < n_here; ++k) {
        const uint32_t opc = uint32_t(__builtin_amdgcn_readlane(int(cw.x), int(k)));
        const uint32_t meta = uint32_t(__builtin_amdgcn_readlane(int(cw.y), int(k)));
        const uint32_t idx = meta & SR_M_INDEX;  // feature / stack slot / constant slot
        // a constant operand: its value (wave-uniform) and its one-hot tangent e_{idx-k0}
        auto const_val = [&]() __attribute__((always_inline)) -> T {
          return idx < 64u ? sr_readlane_val<T>(cval0, idx) : sr_readlane_val<T>(cval1, idx - 64u);
        };
        const int jj = int(idx) - int(k0);
        const T* xrow = xs + size_t(idx) * TROWS + ro + lane;
        const T* sp = my_stk + size_t(idx) * NV * R * 64;
        auto push = [&]() __attribute__((always_inline)) {
          T* pp = my_stk + size_t(((meta >> SR_M_PUSH_SHIFT) & 0x3fu) - 1u) * NV * R * 64;
#pragma unroll
          for (int j = 0; j < R; ++j) {
            pp[j * 64] = v[j];
#pragma unroll
            for (int q = 0; q < KT; ++q) pp[((q + 1) * R + j) * 64] = dv[j][q];
          }
        };
        // r = op(a, b) and its tangents dr = pa da + pb db (pa, pb: the partials) for one of the
        // BASIC binaries with the operand variant known at compile time (round 5: one flat dispatch
        // per instruction instead of decoding the variant; the operand's tangent is known zero for a
        // feature and one-hot for a constant, so those products are not computed).  Every value is
        // the one the general form fma(pa, da, pb db) gives: a product by an exact 0 or 1 and a sum
        // with an exact 0 are exact (up to the sign of a zero, which the gradient sums cannot see),
        // and the skipped product by the zero tangent is still added as (partial x 0) — NaN when that
        // partial is not finite (a DIV by a tiny feature: r finite, -r / x overflows), as in the
        // general form.
        auto basic_bin = [&](auto op_c, auto var_c) __attribute__((always_inline)) {
          constexpr uint32_t B = decltype(op_c)::value;
          constexpr uint32_t V = decltype(var_c)::value;
          constexpr bool LEFT = V == SR_V_SL || V == SR_V_FL || V == SR_V_CL;  // the operand is a
          constexpr int SRC = (V == SR_V_SL || V == SR_V_SR) ? 0 : ((V == SR_V_FL || V == SR_V_FR) ? 1 : 2);
          T cv = T(0);
          if constexpr (SRC == 2) cv = const_val();
          T fix[R] = {};  // constant operand: the tangent at its own slot jj, from the unscaled dv
          T d0[R] = {};
          const bool hot = SRC == 2 && jj >= 0 && jj < KT;
          if (hot) {
#pragma unroll
            for (int q = 0; q < KT; ++q)
#pragma unroll
              for (int j = 0; j < R; ++j) d0[j] = q == jj ? dv[j][q] : d0[j];
          }
#pragma unroll
          for (int j = 0; j < R; ++j) {
            const T ov = SRC == 0 ? sp[j * 64] : (SRC == 1 ? xrow[j * 64] : cv);
            const T av = LEFT ? ov : v[j], bv = LEFT ? v[j] : ov;
            const T rv = sr_binary<T>(B, av, bv);
            T pa, pbv;
            if constexpr (B == SR_B_DIV) {  // d/da = 1/b, d/db = -(a/b)/b = -r (1/b): one division fewer
              pa = T(1) / bv;
              pbv = -rv * pa;
            } else {
              sr_binary_partials<T>(B, av, bv, rv, &pa, &pbv);
            }
            v[j] = rv;
            if constexpr (SRC == 0) {  // stack operand: its tangents from the slot
#pragma unroll
              for (int q = 0; q < KT; ++q) {
                const T od = sp[((q + 1) * R + j) * 64];
                if constexpr (B == SR_B_ADD) {
                  dv[j][q] = LEFT ? od + dv[j][q] : dv[j][q] + od;
                } else if constexpr (B == SR_B_SUB) {
                  dv[j][q] = LEFT ? od - dv[j][q] : dv[j][q] - od;
                } else {
                  dv[j][q] = LEFT ? __builtin_fma(pa, od, pbv * dv[j][q]) : __builtin_fma(pa, dv[j][q], pbv * od);
                }
              }
            } else {
              // feature (zero tangent) or constant (one-hot at jj): every slot is the tos tangent
              // scaled by its own partial; a constant's own slot adds the constant's partial
              if (SRC == 2 && hot) fix[j] = LEFT ? pa + pbv * d0[j] : __builtin_fma(pa, d0[j], pbv);
              if constexpr (B == SR_B_ADD) {
                // scale 1: unchanged
              } else if constexpr (B == SR_B_SUB) {
                if constexpr (LEFT) {
#pragma unroll
                  for (int q = 0; q < KT; ++q) dv[j][q] = -dv[j][q];
                }
              } else {
                const T sc = LEFT ? pbv : pa;
                const T z = (LEFT ? pa : pbv) * T(0);  // (the zero-tangent operand's product)
#pragma unroll
                for (int q = 0; q < KT; ++q) dv[j][q] = __builtin_fma(sc, dv[j][q], z);
              }
            }
          }
          if (SRC == 2 && hot) {
#pragma unroll
            for (int q = 0; q < KT; ++q)
#pragma unroll
              for (int j = 0; j < R; ++j) dv[j][q] = q == jj ? fix[j] : dv[j][q];
          }
        };
        switch (opc) {
          case SR_OP_LOAD_FEAT_PUSH:
            push();
            [[fallthrough]];
          case SR_OP_LOAD_FEAT:
#pragma unroll
            for (int j = 0; j < R; ++j) {
              v[j] = xrow[j * 64];
#pragma unroll
              for (int q = 0; q < KT; ++q) dv[j][q] = T(0);
            }
            break;
          case SR_OP_LOAD_CONST_PUSH:
            push();
            [[fallthrough]];
          case SR_OP_LOAD_CONST: {
            const T cv = const_val();
#pragma unroll
            for (int j = 0; j < R; ++j) {
              v[j] = cv;
#pragma unroll
              for (int q = 0; q < KT; ++q) dv[j][q] = q == jj ? T(1) : T(0);
            }
            break;
          }
#define SR_GRAD_BCASE(B)                                                                                  \
  case SR_BIN_OPC(B, SR_V_SL): basic_bin(std::integral_constant<uint32_t, B>{}, std::integral_constant<uint32_t, SR_V_SL>{}); break; \
  case SR_BIN_OPC(B, SR_V_SR): basic_bin(std::integral_constant<uint32_t, B>{}, std::integral_constant<uint32_t, SR_V_SR>{}); break; \
  case SR_BIN_OPC(B, SR_V_FL): basic_bin(std::integral_constant<uint32_t, B>{}, std::integral_constant<uint32_t, SR_V_FL>{}); break; \
  case SR_BIN_OPC(B, SR_V_FR): basic_bin(std::integral_constant<uint32_t, B>{}, std::integral_constant<uint32_t, SR_V_FR>{}); break; \
  case SR_BIN_OPC(B, SR_V_CL): basic_bin(std::integral_constant<uint32_t, B>{}, std::integral_constant<uint32_t, SR_V_CL>{}); break; \
  case SR_BIN_OPC(B, SR_V_CR): basic_bin(std::integral_constant<uint32_t, B>{}, std::integral_constant<uint32_t, SR_V_CR>{}); break;
          SR_GRAD_BCASE(SR_B_ADD)
          SR_GRAD_BCASE(SR_B_SUB)
          SR_GRAD_BCASE(SR_B_MUL)
          SR_GRAD_BCASE(SR_B_DIV)
#undef SR_GRAD_BCASE
          default:
            if (opc < SR_OP_BINARY0) {
              const uint32_t u = opc >= SR_OP_UNARY_INF0 ? opc - SR_OP_UNARY_INF0 : opc - SR_OP_UNARY0;
              // value and derivative rows: the BASIC operators with the loss kernel's own row bodies
              // (sr_unary_rows: the same values), the rest through the noinline row callees
              // (fused unaries: complete trees have finite inner values, so INFSUB never fires)
              T dfx[R];
              switch (u) {
                case SR_U_NEG:
#pragma unroll
                  for (int j = 0; j < R; ++j) {
                    v[j] = -v[j];
                    dfx[j] = T(-1);
                  }
                  break;
                case SR_U_SQUARE:
#pragma unroll
                  for (int j = 0; j < R; ++j) {
                    const T x = v[j];
                    v[j] = x * x;
                    dfx[j] = T(2) * x;
                  }
                  break;
                case SR_U_CUBE:
#pragma unroll
                  for (int j = 0; j < R; ++j) {
                    const T x = v[j];
                    v[j] = x * x * x;
                    dfx[j] = T(3) * x * x;
                  }
                  break;
                case SR_U_ABS:
#pragma unroll
                  for (int j = 0; j < R; ++j) {
                    const T x = v[j];
                    v[j] = sr_unary<T>(SR_U_ABS, x);
                    dfx[j] = sr_unary_deriv<T>(SR_U_ABS, x, v[j]);
                  }
                  break;
                case SR_U_SQRT:
#pragma unroll
                  for (int j = 0; j < R; ++j) {
                    v[j] = sr_unary<T>(SR_U_SQRT, v[j]);
                    dfx[j] = T(0.5) / v[j];
                  }
                  break;
                case SR_U_EXP:
                  sr_unary_rows<T, SR_U_EXP, R>(v);
#pragma unroll
                  for (int j = 0; j < R; ++j) dfx[j] = v[j];
                  break;
                case SR_U_LOG:
#pragma unroll
                  for (int j = 0; j < R; ++j) dfx[j] = T(1) / v[j];
                  sr_unary_rows<T, SR_U_LOG, R>(v);
                  break;
                case SR_U_COS:
#pragma unroll
                  for (int j = 0; j < R; ++j) dfx[j] = v[j];
                  sr_unary_rows<T, SR_U_COS, R>(v);
                  sr_unary_rows<T, SR_U_SIN, R>(dfx);
#pragma unroll
                  for (int j = 0; j < R; ++j) dfx[j] = -dfx[j];
                  break;
                case SR_U_SIN:
#pragma unroll
                  for (int j = 0; j < R; ++j) dfx[j] = v[j];
                  sr_unary_rows<T, SR_U_SIN, R>(v);
                  sr_unary_rows<T, SR_U_COS, R>(dfx);
                  break;
                default: {
                  SrGVec<T, R> x, y;
#pragma unroll
                  for (int j = 0; j < R; ++j) x[j] = v[j];
                  y = sr_grad_unary_val<T, R>(u, x);
                  x = sr_grad_unary_der<T, R>(u, x, y);
#pragma unroll
                  for (int j = 0; j < R; ++j) {
                    v[j] = y[j];
                    dfx[j] = x[j];
                  }
                  break;
                }
              }
#pragma unroll
              for (int j = 0; j < R; ++j) {
#pragma unroll
                for (int q = 0; q < KT; ++q) dv[j][q] = dfx[j] * dv[j][q];
              }
            } else {
              // the other binaries: value and partials through the row callees, the general tangent form
              const uint32_t b = (opc - SR_OP_BINARY0) / 6u + 1u;
              const uint32_t variant = (opc - SR_OP_BINARY0) % 6u;
              const bool left = variant == SR_V_SL || variant == SR_V_FL || variant == SR_V_CL;
              const bool from_feat = variant == SR_V_FL || variant == SR_V_FR;
              const bool from_stack = variant == SR_V_SL || variant == SR_V_SR;
              const T cv = (!from_feat && !from_stack) ? const_val() : T(0);
              auto operand = [&](int j, T& ov, T (&od)[KT]) {
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
              };
              auto tangents = [&](int j, T pa, T pbv, const T (&od)[KT]) {
                if (left) {
#pragma unroll
                  for (int q = 0; q < KT; ++q) dv[j][q] = __builtin_fma(pa, od[q], pbv * dv[j][q]);
                } else {
#pragma unroll
                  for (int q = 0; q < KT; ++q) dv[j][q] = __builtin_fma(pa, dv[j][q], pbv * od[q]);
                }
              };
              SrGVec<T, R> av, bv;
#pragma unroll
              for (int j = 0; j < R; ++j) {
                T ov, od[KT];
                operand(j, ov, od);
                av[j] = left ? ov : v[j];
                bv[j] = left ? v[j] : ov;
              }
              const SrGVec<T, R> rv = sr_grad_binary_val<T, R>(b, av, bv);
              const SrGVec<T, R> pa = sr_grad_binary_der<T, R, 0>(b, av, bv, rv);
              const SrGVec<T, R> pbv = sr_grad_binary_der<T, R, 1>(b, av, bv, rv);
#pragma unroll
              for (int j = 0; j < R; ++j) {
                T ov, od[KT];
                operand(j, ov, od);
                v[j] = rv[j];
                tangents(j, pa[j], pbv[j], od);
              }
            }
            break;
        }
      }
    }
    // d loss / d constant: (d loss / d pred) * d pred / d constant, padded rows excluded
    T coefs[R];
    if (a.loss_kind == SR_LOSS_L2) {
#pragma unroll
      for (int j = 0; j < R; ++j) coefs[j] = sr_elem_loss_deriv<T>(SR_LOSS_L2, v[j], ys[ro + j * 64 + lane], T(0));
    } else {
      SrGVec<T, R> pv, yv;
#pragma unroll
      for (int j = 0; j < R; ++j) {
        pv[j] = v[j];
        yv[j] = ys[ro + j * 64 + lane];
      }
      pv = sr_grad_loss_der<T, R>(a.loss_kind, pv, yv, a.loss_param);
#pragma unroll
      for (int j = 0; j < R; ++j) coefs[j] = pv[j];
    }
#pragma unroll
    for (int j = 0; j < R; ++j) {
      const int r = j * 64 + lane;
      T coef = coefs[j];
      if (weighted) coef *= wsv[ro + r];
      if (row0 + r >= a.n_rows) coef = T(0);
#pragma unroll
      for (int q = 0; q < KT; ++q) acc[q] = __builtin_fma(double(coef), double(dv[j][q]), acc[q]);
    }
    }  // sub-passes
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

// Launch with `rows` rows per lane: the kernels exist for the bucket's default (sr_grad_rows_per_lane),
// its halves down to 2, and 1 (sr_grad_launch_rows picks one; results do not depend on it: the row
// blocks cover the same rows whatever the rows per lane, see sr_capi.cpp eval_grad_impl).
template <typename T, bool GATHER, int KT, int RR>
hipError_t sr_launch_grad_rows_from(const SrGradArgs<T>& a, int rows, int n_blocks, hipStream_t s) {
  if (rows == RR) return sr_launch_grad<T, KT, 4, GATHER, RR>(a, n_blocks, s);
  if constexpr (RR > 1) return sr_launch_grad_rows_from<T, GATHER, KT, RR / 2>(a, rows, n_blocks, s);
  return hipErrorInvalidValue;
}

template <typename T>
hipError_t sr_launch_grad_any(const SrGradArgs<T>& a, int kt, bool gather, int rows, int n_blocks, hipStream_t s) {
  auto go = [&](auto g) -> hipError_t {
    constexpr bool G = decltype(g)::value;
    switch (kt) {
      case 1: return sr_launch_grad_rows_from<T, G, 1, sr_grad_rows_per_lane(1)>(a, rows, n_blocks, s);
      case 2: return sr_launch_grad_rows_from<T, G, 2, sr_grad_rows_per_lane(2)>(a, rows, n_blocks, s);
      case 4: return sr_launch_grad_rows_from<T, G, 4, sr_grad_rows_per_lane(4)>(a, rows, n_blocks, s);
      case 8: return sr_launch_grad_rows_from<T, G, 8, sr_grad_rows_per_lane(8)>(a, rows, n_blocks, s);
      case 16: return sr_launch_grad_rows_from<T, G, 16, sr_grad_rows_per_lane(16)>(a, rows, n_blocks, s);
      default: return hipErrorInvalidValue;
    }
  };
  return gather ? go(std::true_type{}) : go(std::false_type{});
}
