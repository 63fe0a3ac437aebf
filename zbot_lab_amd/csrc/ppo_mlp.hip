// ppo_mlp.hip — the PPO minibatch update of rsl_rl's ActorCritic as fp32 MFMA kernels for gfx950
// (libzbot_ppo.so, C ABI include/zbot_ppo.h). Restates zbot_lab_amd/rl/ppo.py:PPO.update_steps
// (rsl_rl PPO, reference agents/rsl_rl_ppo_cfg.py:65-91, ppo_learning_notes.md:521-548) per
// minibatch in a handful of launches instead of ~150 torch kernels:
//
//   k_pack       padded / transposed / lane-ordered weight images in the workspace
//   k_rows_reg   (the shipped net shapes) one wave per 16 minibatch rows, activations in registers:
//                gather through the permutation, actor forward (Linear + ELU on
//                v_mfma_f32_16x16x4_f32, the previous layer's accumulators as the B operand, weights
//                shared by the workgroup's four waves through LDS), Gaussian log-prob / KL / clipped
//                surrogate and its gradient, actor backward dX; then the critic forward, clipped value
//                loss and backward. Every layer's input X_l and pre-activation gradient dZ_l go to HBM
//                (octet-blocked rows) for the weight gradients.
//   k_rows       the same with the activations in LDS (32-row tiles; any other shape, ZBP_ROWS=lds)
//   k_wgrad      dW_l = dZ_l^T X_l and db_l = sum dZ_l: an LDS-tiled GEMM over the minibatch rows,
//                128 x 128 output blocks, split-K over row ranges sized to one round of the device's
//                resident workgroups; partial tiles to the workspace
//   k_reduce     partial tiles -> every parameter's .grad, the std gradient, the minibatch stats
//
// and, on one GPU, k_adam (adaptive learning rate, global-norm clipping from k_reduce's per-tile sums
// of squares, or k_norm's, Adam) + the re-pack (k_pack, which also writes the new rate and step); the rollout's policy step (k_act_reg / k_act), its bookkeeping (k_env_post) and
// GAE (k_gae, k_adv_stats, k_adv_norm). Exact fp32 throughout (the MFMA is a k-ordered fmaf chain);
// results differ from torch's only by summation order. MI355X mapping: the weights (<= 450 KB per
// net) stay L2-resident; design and measurements in DESIGN.md §7 (round 5).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "zbot_ppo.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));
constexpr int TR = 32;            // rows per tile (the MFMA's M)
constexpr int MAXL = ZBP_MAX_LAYERS;
constexpr int PART = 32 * 32 + 32;  // one weight-gradient partial tile + its bias column
constexpr int NSTAT = 16;           // per-row-tile partial sums (surrogate, value, kl, std grads)
// k_rows workgroup: 8 waves on one 32-row tile (a layer's output tiles dealt over them): with the
// C5 nets' 97 KB of activations one workgroup fits a CU, so two waves share each SIMD and cover each
// other's LDS / L2 waits
constexpr int ROW_THREADS = 512;

thread_local char g_err[256] = "";
int fail(int code, const char* what) {
  snprintf(g_err, sizeof(g_err), "%s", what);
  return code;
}
int hip_fail(hipError_t e, const char* what) {
  snprintf(g_err, sizeof(g_err), "%s: %s", what, hipGetErrorString(e));
  return -2;
}

inline int pad32(int d) { return (d + 31) & ~31; }

// Row buffers (X_l, dZ_l) in HBM are octet-blocked feature-major: feature f of minibatch row i of a
// P-feature buffer at ((i >> 3) P + f) 8 + (i & 7), i.e. for every octet of rows the features' 8-row
// runs (32 B) back to back. k_wgrad's lanes (one feature each, four rows) then read 1 KB contiguous
// per instruction (8 full lines) instead of one 16-byte piece from each of 32 lines.
__host__ __device__ __forceinline__ int64_t rbo(int P, int f, int i) { return ((int64_t)(i >> 3) * P + f) * 8 + (i & 7); }

// one net in the workspace: dims and float offsets of its images and row buffers
struct NetW {
  int L, d[MAXL + 1], p[MAXL + 1];
  int64_t wp[MAXL], wt[MAXL], bp[MAXL];  // padded weights [p(l+1)][p(l)], transposed [p(l)][p(l+1)], bias [p(l+1)]
  int64_t wr[MAXL], wtr[MAXL];           // the same in k_rows_reg's lane order (forward / backward A operands)
  int64_t x[MAXL], dz[MAXL];             // row buffers: X_l [B][p(l)], dZ_l [B][p(l+1)]
};
struct Layout {
  NetW n[2];
  int64_t stats;  // [tiles][NSTAT] per-row-tile partial sums
  int64_t part;   // [splits (the largest)][wtiles][PART] weight-gradient partials
  int wtiles, tile0[2 * MAXL + 1];  // weight tiles of (net, layer) in order, prefix counts
  int ngroups, grp0[2 * MAXL + 1];  // k_wgrad workgroups (<= 4 x 4 output x reduction tiles) of (net, layer), prefix counts
  int splits;                       // the largest row split count
  int sp_nl[2 * MAXL];              // row splits of (net, layer) (one count for all, see make_layout)
  int ord[2 * MAXL];                // k_wgrad launch order of the (net, layer)s
  int blk0[2 * MAXL + 1];           // k_wgrad launch: first workgroup of the (net, layer) at order position i
  int64_t scratch;  // [max(64, wtiles + 1)] gradient sums of squares: k_norm's per block, or k_reduce's per weight tile
  int64_t rng;      // [1] uint32: the draw counter of the in-kernel action noise, advanced by every k_pack
  int64_t total;
};

// k_wgrad workgroups resident at once: two per CU (64 KB of LDS each); the CU count of the current
// device (256 on MI355X; 256 when no device is visible)
int wgrad_slots() {
  static const int cus = [] {
    int d = 0, n = 0;
    if (hipGetDevice(&d) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d) != hipSuccess ||
        n <= 0)
      n = 256;
    (void)hipGetLastError();
    return n;
  }();
  // (ZBP_WGRAD_SLOTS_PER_CU, read once: the split-K A/B; default 2 = the resident k_wgrad workgroups)
  static const int per_cu = [] {
    const char* e = getenv("ZBP_WGRAD_SLOTS_PER_CU");
    const int v = e ? atoi(e) : 2;
    return v >= 1 && v <= 8 ? v : 2;
  }();
  return per_cu * cus;
}

Layout make_layout(const zbp_net* a, const zbp_net* c, int B) {
  Layout lo{};
  int64_t off = 0;
  auto take = [&](int64_t n) { int64_t o = off; off += (n + 63) & ~int64_t(63); return o; };
  const zbp_net* nets[2] = {a, c};
  int t = 0;
  for (int k = 0; k < 2; ++k) {
    NetW& w = lo.n[k];
    w.L = nets[k]->n_layers;
    for (int l = 0; l <= w.L; ++l) { w.d[l] = nets[k]->dim[l]; w.p[l] = pad32(w.d[l]); }
    for (int l = 0; l < w.L; ++l) {
      w.wp[l] = take((int64_t)w.p[l + 1] * w.p[l]);
      w.wt[l] = take((int64_t)w.p[l] * w.p[l + 1]);
      w.bp[l] = take(w.p[l + 1]);
      w.wr[l] = take((int64_t)w.p[l + 1] * w.p[l]);
      w.wtr[l] = take((int64_t)w.p[l] * w.p[l + 1]);
      w.x[l] = take((int64_t)B * w.p[l]);
      w.dz[l] = take((int64_t)B * w.p[l + 1]);
      lo.tile0[k * MAXL + l] = t;
      t += (w.p[l + 1] / 32) * (w.p[l] / 32);
    }
    for (int l = w.L; l < MAXL; ++l) lo.tile0[k * MAXL + l] = t;
  }
  lo.tile0[2 * MAXL] = t;
  lo.wtiles = t;
  // weight-gradient workgroups: per (net, layer) groups of up to 4 output tiles (one wave each) x up
  // to 4 reduction tiles
  int g = 0;
  for (int k = 0; k < 2; ++k)
    for (int l = 0; l < MAXL; ++l) {
      lo.grp0[k * MAXL + l] = g;
      if (l < lo.n[k].L) g += ((lo.n[k].p[l + 1] / 32 + 3) / 4) * ((lo.n[k].p[l] / 32 + 3) / 4);
    }
  lo.grp0[2 * MAXL] = g;
  lo.ngroups = g;
  lo.stats = take((int64_t)(B / 16) * NSTAT);  // (per 32-row tile of k_rows, per 16-row wave of k_rows_reg)
  // row splits of the weight gradients: as many as fill the device's resident k_wgrad workgroups in
  // ONE round (groups x splits <= slots; a second, partly filled round would leave most CUs idle for
  // a whole split's time); a split is a contiguous range of 32-row chunks (k_wgrad's LDS chunks). The
  // same count for every layer: a chunk costs about the same in every group (its copy and barrier
  // latency, not the MFMAs, set the pace: splits weighted by the groups' MFMA work made the launch
  // 66 -> 87 us)
  const int C = B / 32;
  int s = wgrad_slots() / g;
  s = s < 1 ? 1 : (s > C ? C : (s > 1024 ? 1024 : s));
  // launch order: the layers whose blocks keep all four waves' MFMAs busy (2 x 2 tiles per wave)
  // first, then the input / output layers (half the MFMAs per wave): with the launch filling every CU's
  // first slot before its second, a CU then pairs a busy block with a light one instead of two busy ones
  int b = 0, pos = 0;
  for (int pass = 0; pass < 2; ++pass)
    for (int nl = 0; nl < 2 * MAXL; ++nl) {
      const int k = nl / MAXL, l = nl % MAXL;
      const bool busy = l < lo.n[k].L && lo.n[k].p[l + 1] >= 64 && lo.n[k].p[l] >= 64;
      if ((pass == 0) != busy) continue;
      lo.ord[pos] = nl;
      lo.blk0[pos++] = b;
      lo.sp_nl[nl] = s;
      b += (lo.grp0[nl + 1] - lo.grp0[nl]) * s;
    }
  lo.blk0[2 * MAXL] = b;
  lo.splits = s;
  lo.part = take((int64_t)s * t * PART);
  lo.scratch = take(t + 1 > 64 ? t + 1 : 64);
  lo.rng = take(1);
  lo.total = off;
  return lo;
}

const char* check_net(const zbp_net* n) {
  if (!n || n->n_layers < 1 || n->n_layers > MAXL) return "n_layers must be 1..4";
  if (n->dim[0] < 1 || n->dim[0] > 32) return "input dim must be 1..32";
  for (int l = 1; l < n->n_layers; ++l)
    if (n->dim[l] < 32 || n->dim[l] > 256 || n->dim[l] % 32) return "hidden dims must be multiples of 32 up to 256";
  if (n->dim[n->n_layers] < 1 || n->dim[n->n_layers] > 32) return "output dim must be 1..32";
  for (int l = 0; l < n->n_layers; ++l)
    if (!n->w[l] || !n->b[l]) return "null weight / bias";
  return nullptr;
}

__device__ __forceinline__ f32x16 mfma(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

// C[32 rows][32 cols] = sum_k A[r][k] B[k][c] over k < kp (kp a multiple of 32): A row-major in LDS
// (row stride sa floats), B given as the 32 rows m[(c0 + c) * ldm + k] of a row-major global matrix
// (the reduction index contiguous, L2-resident). Lane (c = lane & 31, h = lane >> 5) feeds
// A[c][.] / B[.][c] on the reduction indices [h kp / 2, (h + 1) kp / 2) (the MFMA's k = 0 / 1
// halves). The B stream runs 16 MFMAs (four float4) ahead of its use: one wave per SIMD has no
// other wave to cover an L2 round trip.
__device__ __forceinline__ f32x16 tile_mma(const float* __restrict__ a, int sa, const float* __restrict__ m, int ldm,
                                           int kp, int c0) {
  const int lane = threadIdx.x & 63, c = lane & 31, h = lane >> 5, half = kp >> 1;
  const float* ar = a + c * sa + h * half;
  const float4* br = reinterpret_cast<const float4*>(m + (int64_t)(c0 + c) * ldm + h * half);
  const int nq = half >> 2;  // float4 steps (>= 4)
  f32x16 acc = {};
  float4 b0 = br[0], b1 = br[1], b2 = br[2], b3 = br[3];
  for (int q = 0; q < nq; q += 4) {
    const float4 a0 = *reinterpret_cast<const float4*>(ar + 4 * q);
    const float4 a1 = *reinterpret_cast<const float4*>(ar + 4 * q + 4);
    const float4 a2 = *reinterpret_cast<const float4*>(ar + 4 * q + 8);
    const float4 a3 = *reinterpret_cast<const float4*>(ar + 4 * q + 12);
    const float4 u0 = b0, u1 = b1, u2 = b2, u3 = b3;
    if (q + 4 < nq) { b0 = br[q + 4]; b1 = br[q + 5]; b2 = br[q + 6]; b3 = br[q + 7]; }
    acc = mfma(a0.x, u0.x, acc); acc = mfma(a0.y, u0.y, acc); acc = mfma(a0.z, u0.z, acc); acc = mfma(a0.w, u0.w, acc);
    acc = mfma(a1.x, u1.x, acc); acc = mfma(a1.y, u1.y, acc); acc = mfma(a1.z, u1.z, acc); acc = mfma(a1.w, u1.w, acc);
    acc = mfma(a2.x, u2.x, acc); acc = mfma(a2.y, u2.y, acc); acc = mfma(a2.z, u2.z, acc); acc = mfma(a2.w, u2.w, acc);
    acc = mfma(a3.x, u3.x, acc); acc = mfma(a3.y, u3.y, acc); acc = mfma(a3.z, u3.z, acc); acc = mfma(a3.w, u3.w, acc);
  }
  return acc;
}
// row / column of accumulator register r of a 32x32 MFMA tile in this lane: registers 4q .. 4q + 3
// hold rows 8q + 4h .. 8q + 4h + 3 of column lane & 31
__device__ __forceinline__ int acc_row(int r) { return (r & 3) + 8 * (r >> 2) + 4 * ((threadIdx.x & 63) >> 5); }
__device__ __forceinline__ int acc_col() { return threadIdx.x & 31; }

// ------------------------------------------------------------------------------- k_pack
struct PackArgs {
  NetW n[2];
  const float* w[2][MAXL];
  const float* b[2][MAXL];
  float* ws;
  // zbp_optimizer_step's tail (tail != 0; one thread): the new learning rate and step counter, which
  // every k_adam workgroup read as the old ones (so written after that launch), and the loss sums
  int tail, n_params;
  float* lr;
  const float* stats;
  float* acc;
  float desired_kl;
  float* step[ZBP_MAX_PARAMS];
  uint32_t* rng;  // the workspace's noise draw counter: +1 per launch (one thread)
};
__device__ __forceinline__ float adaptive_lr(float lr, float kl, float desired_kl) {
  // rsl_rl's adaptive schedule on the minibatch KL
  if (desired_kl > 0.f) {
    if (kl > desired_kl * 2.f) lr = fmaxf(lr / 1.5f, 1e-5f);
    else if (kl > 0.f && kl < desired_kl / 2.f) lr = fminf(lr * 1.5f, 1e-2f);
  }
  return lr;
}
__global__ void k_pack(PackArgs A) {
  if (blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0) *A.rng += 1u;
  if (A.tail && blockIdx.x == 0 && blockIdx.y == 0 && blockIdx.z == 0 && threadIdx.x == 0) {
    *A.lr = adaptive_lr(*A.lr, A.stats[0], A.desired_kl);
    const float step = A.step[0][0] + 1.f;
    for (int t = 0; t < A.n_params; ++t) A.step[t][0] = step;
    A.acc[0] += A.stats[1];
    A.acc[1] += A.stats[2];
    A.acc[2] += A.stats[3];
  }
  const int net = blockIdx.y, l = blockIdx.z;
  const NetW& w = A.n[net];
  if (l >= w.L) return;
  const int P0 = w.p[l], P1 = w.p[l + 1], D0 = w.d[l], D1 = w.d[l + 1];
  float* wp = A.ws + w.wp[l];
  float* wt = A.ws + w.wt[l];
  float* wr = A.ws + w.wr[l];
  float* wtr = A.ws + w.wtr[l];
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < P0 * P1; e += gridDim.x * blockDim.x) {
    const int n = e / P0, k = e % P0;
    const float v = (n < D1 && k < D0) ? A.w[net][l][n * D0 + k] : 0.f;
    wp[e] = v;
    wt[k * P1 + n] = v;
    // k_rows_reg's A operands (v_mfma_f32_16x16x4_f32): 16 x 16 blocks in its order (reduction
    // tile outer, output tile inner); in a block, lane (output index & 15) + 16 g holds the four
    // reduction indices 4 g + u as one float4 (a block is one contiguous KB: conflict-free
    // ds_read_b128 from the LDS copy)
    {
      const int T1h = P1 / 16, T0h = P0 / 16;
      wr[(int64_t)((k >> 4) * T1h + (n >> 4)) * 256 + ((n & 15) + 16 * ((k >> 2) & 3)) * 4 + (k & 3)] = v;
      wtr[(int64_t)((n >> 4) * T0h + (k >> 4)) * 256 + ((k & 15) + 16 * ((n >> 2) & 3)) * 4 + (n & 3)] = v;
    }
  }
  if (blockIdx.x == 0)
    for (int n = threadIdx.x; n < P1; n += blockDim.x) A.ws[w.bp[l] + n] = n < D1 ? A.b[net][l][n] : 0.f;
}

// ------------------------------------------------------------------------------- k_rows
// Row buffers in HBM are feature-major (X_l [p(l)][B], dZ_l [p(l+1)][B]): a row tile writes whole
// 128-byte lines (32 rows of one feature) as float4 quads of rows, and k_wgrad streams float4 quads
// of rows per lane. In LDS the tile's activations are row-major [32][P + 4]; the backward pass
// writes dZ_{l-1} over X_l in place (each element read once by the thread that overwrites it).
struct RowArgs {
  NetW n[2];
  zbp_batch bt;
  zbp_loss_cfg lc;
  const float* std_param;
  float* ws;
  int64_t stats;
  int B;
  int lds_x[MAXL], lds_dz, lds_out, lds_red;  // LDS float offsets
};

// forward through one net for the row tile; the output layer's pre-activations land in `out`
// ([32][33]). kStore: every hidden layer's input X_l also goes to the HBM row buffers (feature-major,
// B rows) for the weight gradients; the rollout's forward (k_act) keeps them in LDS only.
template <bool kStore>
__device__ void net_forward_t(const NetW& w, float* ws, int B, const int* lds_x, int lds_out, float* lds, int row0) {
  const int wave = threadIdx.x >> 6, h = (threadIdx.x & 63) >> 5, nw = blockDim.x >> 6;
  for (int l = 0; l < w.L; ++l) {
    const int P0 = w.p[l], P1 = w.p[l + 1];
    const bool last = l == w.L - 1;
    const float* xs = lds + lds_x[l];
    const float* wp = ws + w.wp[l];
    const float* bp = ws + w.bp[l];
    for (int t = wave; t < P1 / 32; t += nw) {
      const f32x16 acc = tile_mma(xs, P0 + 4, wp, P0, P0, 32 * t);
      const int n = 32 * t + acc_col();
      const float bias = bp[n];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = 8 * q + 4 * h + u;
          v[u] = acc[4 * q + u] + bias;
          if (last) {
            lds[lds_out + i * 33 + n] = v[u];
          } else {
            v[u] = v[u] > 0.f ? v[u] : expf(v[u]) - 1.f;  // ELU(alpha = 1), as ATen's elu kernel
            lds[lds_x[l + 1] + i * (P1 + 4) + n] = v[u];
          }
        }
        if (kStore && !last)
          *reinterpret_cast<float4*>(ws + w.x[l + 1] + rbo(P1, n, row0 + 8 * q + 4 * h)) =
              make_float4(v[0], v[1], v[2], v[3]);
      }
    }
    __syncthreads();
  }
}
__device__ void net_forward(const RowArgs& A, const NetW& w, float* lds, int row0) {
  net_forward_t<true>(w, A.ws, A.B, A.lds_x, A.lds_out, lds, row0);
}

// backward through one net from dZ of the output layer (lds_dz, [32][p(L) + 4])
__device__ void net_backward(const RowArgs& A, const NetW& w, float* lds, int row0) {
  const int wave = threadIdx.x >> 6, h = (threadIdx.x & 63) >> 5, nw = blockDim.x >> 6;
  for (int l = w.L - 1; l >= 1; --l) {
    const int P0 = w.p[l], P1 = w.p[l + 1];
    const float* dz = lds + (l == w.L - 1 ? A.lds_dz : A.lds_x[l + 1]);
    float* xs = lds + A.lds_x[l];  // X_l, overwritten by dZ_{l-1}
    const float* wt = A.ws + w.wt[l];
    for (int t = wave; t < P0 / 32; t += nw) {
      const f32x16 acc = tile_mma(dz, P1 + 4, wt, P1, P1, 32 * t);
      const int k = 32 * t + acc_col();
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float g[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int i = 8 * q + 4 * h + u;
          const float x = xs[i * (P0 + 4) + k];
          g[u] = acc[4 * q + u] * (x > 0.f ? 1.f : x + 1.f);  // ELU'(z) = exp(z) = x + 1 for z <= 0
          xs[i * (P0 + 4) + k] = g[u];
        }
        *reinterpret_cast<float4*>(A.ws + w.dz[l - 1] + rbo(P0, k, row0 + 8 * q + 4 * h)) =
            make_float4(g[0], g[1], g[2], g[3]);
      }
    }
    __syncthreads();
  }
}

// gather the tile's input rows (obs or critic obs) into X_0 (LDS + HBM), zero-padded
__device__ void gather_input(const RowArgs& A, const NetW& w, const float* src, int dim, float* lds, int row0) {
  const int P0 = w.p[0];
  for (int e = threadIdx.x; e < TR * P0; e += blockDim.x) {
    const int k = e / TR, i = e % TR;
    const int64_t row = A.bt.idx[A.bt.idx_offset + row0 + i];
    const float v = k < dim ? src[row * dim + k] : 0.f;
    lds[A.lds_x[0] + i * (P0 + 4) + k] = v;
    A.ws[w.x[0] + rbo(P0, k, row0 + i)] = v;
  }
  __syncthreads();
}

__device__ __forceinline__ float wave_sum(float v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(ROW_THREADS) void k_rows(RowArgs A) {
  extern __shared__ float lds[];
  const int row0 = blockIdx.x * TR;
  const int tid = threadIdx.x;
  const zbp_batch& bt = A.bt;
  const int NA = bt.num_actions;
  const float invB = 1.f / (float)bt.batch;
  float* red = lds + A.lds_red;  // [NSTAT] per-tile sums
  if (tid < NSTAT) red[tid] = 0.f;

  // ---- actor: forward, Gaussian log-prob, clipped surrogate, KL; dL/dmu into dZ of the output
  const NetW& wa = A.n[0];
  gather_input(A, wa, bt.obs, bt.obs_dim, lds, row0);
  net_forward(A, wa, lds, row0);
  {
    float* dz = lds + A.lds_dz;
    const int Pout = wa.p[wa.L];
    float surr = 0.f, kl = 0.f, sg[NSTAT - 3];
#pragma unroll
    for (int a = 0; a < NSTAT - 3; ++a) sg[a] = 0.f;
    if (tid < TR) {
      const int i = tid;
      const int64_t row = bt.idx[bt.idx_offset + row0 + i];
      const float kLog2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
      float lp = 0.f;
      for (int a = 0; a < NA; ++a) {
        const float mu = lds[A.lds_out + i * 33 + a], s = A.std_param[a];
        const float x = bt.actions[row * NA + a], diff = x - mu;
        lp += -(diff * diff) / (2.f * (s * s)) - logf(s) - kLog2Pi;
        const float os = bt.sigma[row * NA + a], om = bt.mu[row * NA + a];
        kl += logf(s / os + 1e-5f) + (os * os + (om - mu) * (om - mu)) / (2.f * (s * s)) - 0.5f;
      }
      const float adv = bt.advantages[row], clip = A.lc.clip_param;
      const float ratio = expf(lp - bt.log_prob[row]);
      const float rc = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip);
      const float s1 = -adv * ratio, s2 = -adv * rc;
      surr = fmaxf(s1, s2);
      // d max(s1, s2) / d ratio (torch.max splits a tie evenly; clamp passes the gradient inside
      // [1 - clip, 1 + clip], bounds included)
      const float in = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
      const float w1 = s1 > s2 ? 1.f : (s1 < s2 ? 0.f : 0.5f);
      const float g = (w1 * -adv + (1.f - w1) * -adv * in) * ratio * invB;  // dL / dlog_prob
      for (int a = 0; a < Pout; ++a) {
        float d = 0.f;
        if (a < NA) {
          const float mu = lds[A.lds_out + i * 33 + a], s = A.std_param[a];
          const float diff = bt.actions[row * NA + a] - mu;
          d = g * diff / (s * s);
#pragma unroll
          for (int b = 0; b < NSTAT - 3; ++b)
            if (b == a) sg[b] = g * (diff * diff / (s * s * s) - 1.f / s);
        }
        dz[i * (Pout + 4) + a] = d;
        A.ws[wa.dz[wa.L - 1] + rbo(Pout, a, row0 + i)] = d;
      }
    }
    if (tid < 64) {
      surr = wave_sum(surr);
      kl = wave_sum(kl);
#pragma unroll
      for (int a = 0; a < NSTAT - 3; ++a) sg[a] = wave_sum(sg[a]);
      if (tid == 0) {
        red[0] = surr;
        red[2] = kl;
#pragma unroll
        for (int a = 0; a < NSTAT - 3; ++a) red[3 + a] = sg[a];
      }
    }
    __syncthreads();
  }
  net_backward(A, wa, lds, row0);

  // ---- critic: forward, clipped value loss, backward
  const NetW& wc = A.n[1];
  gather_input(A, wc, bt.critic_obs, bt.critic_obs_dim, lds, row0);
  net_forward(A, wc, lds, row0);
  {
    float* dz = lds + A.lds_dz;
    const int Pout = wc.p[wc.L];
    float vl = 0.f;
    if (tid < TR) {
      const int i = tid;
      const int64_t row = bt.idx[bt.idx_offset + row0 + i];
      const float v = lds[A.lds_out + i * 33], tv = bt.values[row], ret = bt.returns[row], clip = A.lc.clip_param;
      float dv;
      if (A.lc.use_clipped_value_loss) {
        const float vd = v - tv;
        const float vc = tv + fminf(fmaxf(vd, -clip), clip);
        const float ea = (v - ret) * (v - ret), ec = (vc - ret) * (vc - ret);
        vl = fmaxf(ea, ec);
        const float wa_ = ea > ec ? 1.f : (ea < ec ? 0.f : 0.5f);
        const float in = (vd >= -clip && vd <= clip) ? 1.f : 0.f;
        dv = wa_ * 2.f * (v - ret) + (1.f - wa_) * 2.f * (vc - ret) * in;
      } else {
        vl = (ret - v) * (ret - v);
        dv = 2.f * (v - ret);
      }
      dv *= A.lc.value_loss_coef * invB;
      for (int a = 0; a < Pout; ++a) {
        dz[i * (Pout + 4) + a] = a == 0 ? dv : 0.f;
        A.ws[wc.dz[wc.L - 1] + rbo(Pout, a, row0 + i)] = a == 0 ? dv : 0.f;
      }
    }
    if (tid < 64) {
      vl = wave_sum(vl);
      if (tid == 0) red[1] = vl;
    }
    __syncthreads();
  }
  net_backward(A, wc, lds, row0);
  if (tid < NSTAT) A.ws[A.stats + (int64_t)blockIdx.x * NSTAT + tid] = red[tid];
}

// ------------------------------------------------------------------------------- k_rows_reg
// k_rows for the shipped net shapes (three hidden layers of 16 T1, 16 T2, 16 T3 units, inputs and
// outputs <= 32: rsl_rl's [128, 128, 128] and the stand-up / v2 [256, 256, 128]), one WAVE per 16-row
// tile and the activations in registers. A layer is the transposed product Z^T = W X^T on
// v_mfma_f32_16x16x4_f32 with the weights as the A operand and the activations as the B operand
// straight from the previous layer's accumulators: an accumulator tile (4 registers) holds, in lane
// (row r = lane & 15, g = lane >> 4), register u, feature 4 g + u of row r -- exactly the B operand
// of 4 MFMAs whose reduction index runs over the tile's 16 features. A 256-wide layer keeps 16 input
// + 16 output tiles (128 registers) live, so two waves share each SIMD and cover each other's
// epilogues (bias, ELU, the row-buffer stores) and memory waits. The workgroup's four waves share
// the weights through LDS (double-buffered 32 KB chunks of 32 blocks, one barrier per chunk). X_l
// and dZ_l go to HBM octet-blocked (rbo) for k_wgrad; the backward pass reads X_l back for ELU'.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef f32x4 Tile;

__device__ __forceinline__ f32x4 mfma16(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ int rr_g() { return (threadIdx.x & 63) >> 4; }
// row buffers (rbo): element (feature 16 o + 4 g + u, row row0 + r) of a P-feature buffer at
// base = buffer + rbo(P, 0, row0) as base[uniform part (16 o + u) 8] + lane part
// ((r >> 3) P 8 + 32 g + (r & 7)): the uniform part stays scalar, the lane part one VGPR offset
__device__ __forceinline__ int rr_lane_off(int P) {
  const int r = threadIdx.x & 15;
  return (r >> 3) * P * 8 + 32 * rr_g() + (r & 7);
}
__device__ __forceinline__ float* rr_base(float* buf, int P, int row0) { return buf + (int64_t)(row0 >> 3) * P * 8; }
__device__ __forceinline__ float* rr_at(float* base, int o, int u) { return base + (16 * o + u) * 8; }

// out[o] = sum_i A(o, i) in[i] over the blocks of a lane-ordered image: block b = (i, o) (reduction
// tile outer: consecutive blocks feed different accumulators) = one float4 per lane, the A operands
// of 4 MFMAs whose B operands are in[i]'s registers, read from the workgroup's LDS copy of the
// current chunk while the next chunk is in flight from L2.
// CB = blocks per chunk: 32 (32 KB chunks, 64 KB of LDS per workgroup: two workgroups per CU) for
// the 256-wide nets; 16 for the 128-wide ones, whose waves fit three to a SIMD (168 registers) and
// whose three workgroups per CU then need 32 KB of LDS each
constexpr int RR_WG = 256;                    // threads per workgroup (4 waves, 4 row tiles)
template <int T1> constexpr int rr_cb() { return T1 <= 8 ? 16 : 32; }
template <int T1> constexpr int rr_occ() { return T1 <= 8 ? 3 : 2; }
template <int CB> using RrStage = float4[CB * 64 / RR_WG];  // this thread's share of a chunk in flight
// chunk `chunk` of an image of NB blocks into the thread's stage registers (zero past the end)
template <int NB, int CB>
__device__ __forceinline__ void rr_fetch(const float* __restrict__ img, int chunk, RrStage<CB>& st) {
  constexpr int NF = NB * 64, PER = CB * 64 / RR_WG;
  const float4* g = reinterpret_cast<const float4*>(img);
#pragma unroll
  for (int m = 0; m < PER; ++m) {
    const int e = chunk * CB * 64 + threadIdx.x + m * RR_WG;
    if (chunk * CB * 64 + m * RR_WG < NF) st[m] = e < NF ? g[e] : float4{};
  }
}
// out[o] = sum_i A(o, i) in[i]; st holds the image's chunk 0 on entry (the caller fetched it, ahead of
// its own epilogue stores: a wait for the weights never waits for those stores to drain)
template <int TI, int TO, int CB>
__device__ __forceinline__ void rr_layer(const float* __restrict__ img, float4* __restrict__ wl, const Tile (&in)[TI],
                                         Tile (&out)[TO], RrStage<CB>& st) {
  constexpr int NB = TI * TO, NC = (NB + CB - 1) / CB;
  constexpr int NF = NB * 64, RR_PER = CB * 64 / RR_WG;
  const int t = threadIdx.x, lane = t & 63;
#pragma unroll
  for (int o = 0; o < TO; ++o) out[o] = Tile{};
#pragma unroll
  for (int m = 0; m < RR_PER; ++m)
    if (m * RR_WG < NF) wl[t + m * RR_WG] = st[m];
  __syncthreads();
  if (NC > 1) rr_fetch<NB, CB>(img, 1, st);
#pragma unroll
  for (int c = 0; c < NC; ++c) {
    const float4* cb = wl + (c & 1) * CB * 64 + lane;
#pragma unroll
    for (int bb = 0; bb < CB; ++bb) {
      const int b = c * CB + bb;
      if (b < NB) {
        const int i = b / TO, o = b % TO;
        const float4 w = cb[bb * 64];
        Tile a = out[o];
        a = mfma16(w.x, in[i][0], a);
        a = mfma16(w.y, in[i][1], a);
        a = mfma16(w.z, in[i][2], a);
        a = mfma16(w.w, in[i][3], a);
        out[o] = a;
      }
    }
    if (c + 1 < NC) {
      float4* nb = wl + ((c + 1) & 1) * CB * 64;
#pragma unroll
      for (int m = 0; m < RR_PER; ++m)
        if ((c + 1) * CB * 64 + m * RR_WG < NF) nb[t + m * RR_WG] = st[m];
    }
    __syncthreads();  // chunk c consumed by every wave, chunk c + 1 in LDS
    if (c + 2 < NC) rr_fetch<NB, CB>(img, c + 2, st);
  }
}

// forward layer l: + bias, ELU (hidden layers: also X_{l+1} to HBM)
// (NBN > 0: the next layer's image `next` has NBN blocks; its chunk 0 is fetched before this epilogue)
template <int TI, int TO, bool kLast, bool kStore, int NBN, int CB>
__device__ __forceinline__ void rr_forward(const NetW& w, int l, float* __restrict__ ws, float4* __restrict__ wl, int row0,
                                           const Tile (&in)[TI], Tile (&out)[TO], RrStage<CB>& st, const float* next) {
  const int lo = rr_lane_off(16 * TO);
  rr_layer<TI, TO, CB>(ws + w.wr[l], wl, in, out, st);
  if (NBN > 0) rr_fetch<NBN, CB>(next, 0, st);
  const float* bp = ws + w.bp[l] + 4 * rr_g();
  float* xb = rr_base(ws + w.x[l + 1], 16 * TO, row0);
#pragma unroll
  for (int o = 0; o < TO; ++o) {
    const float4 bq = *reinterpret_cast<const float4*>(bp + 16 * o);
    const float bv[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v = out[o][u] + bv[u];
      if (!kLast) {
        v = v > 0.f ? v : expf(v) - 1.f;  // ELU(alpha = 1), as ATen's elu kernel
        if (kStore) rr_at(xb, o, u)[lo] = v;
      }
      out[o][u] = v;
    }
  }
}

// backward through layer l >= 1: dZ_{l-1} = (W_l^T dZ_l) * ELU'(X_l), to registers and HBM
template <int TI, int TO, int NBN, int CB>
__device__ __forceinline__ void rr_backward(const NetW& w, int l, float* __restrict__ ws, float4* __restrict__ wl, int row0,
                                            const Tile (&dz)[TI], Tile (&out)[TO], RrStage<CB>& st, const float* next) {
  const int lo = rr_lane_off(16 * TO);
  float* xb = rr_base(ws + w.x[l], 16 * TO, row0);
  float* db = rr_base(ws + w.dz[l - 1], 16 * TO, row0);
  // X_l for ELU': loaded ahead of the product where the registers allow (its latency then hides
  // under the MFMAs; the 256 x 256 layer has no room at two waves per SIMD and loads it after)
  constexpr int NPRE = TI + 2 * TO <= 40 ? TO : TO / 2;  // tiles of X_l loaded ahead
  Tile xl[TO];
#pragma unroll
  for (int o = 0; o < NPRE; ++o)
#pragma unroll
    for (int u = 0; u < 4; ++u) xl[o][u] = rr_at(xb, o, u)[lo];
  rr_layer<TI, TO, CB>(ws + w.wtr[l], wl, dz, out, st);
  if (NBN > 0) rr_fetch<NBN, CB>(next, 0, st);
#pragma unroll
  for (int o = 0; o < TO; ++o)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float x = o < NPRE ? xl[o][u] : rr_at(xb, o, u)[lo];
      const float gr = out[o][u] * (x > 0.f ? 1.f : x + 1.f);  // ELU'(z) = exp(z) = x + 1 for z <= 0
      out[o][u] = gr;
      rr_at(db, o, u)[lo] = gr;
    }
}

// the tile's input rows (through the permutation) as the first layer's B operand, zero-padded to 32
__device__ __forceinline__ void rr_gather(const NetW& w, float* __restrict__ ws, int row0, const float* src, int dim,
                                          int64_t row, Tile (&x)[2]) {
  const int lo = rr_lane_off(32);
  float* xb = rr_base(ws + w.x[0], 32, row0);
  const float* sr = src + row * dim;
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = 16 * o + 4 * rr_g() + u;
      const float v = k < dim ? sr[k] : 0.f;
      x[o][u] = v;
      rr_at(xb, o, u)[lo] = v;
    }
}

__device__ __forceinline__ void rr_store_dz(const NetW& w, float* __restrict__ ws, int row0, const Tile (&d)[2]) {
  const int lo = rr_lane_off(32);
  float* db = rr_base(ws + w.dz[w.L - 1], 32, row0);
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int u = 0; u < 4; ++u) rr_at(db, o, u)[lo] = d[o][u];
}

// sum over the 16 rows of a wave (lanes with the same g)
__device__ __forceinline__ float rr_row_sum(float v) {
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o);
  return v;
}
// sum over the 4 feature groups of a row (lanes r, r + 16, r + 32, r + 48)
__device__ __forceinline__ float rr_feat_sum(float v) {
  v += __shfl_xor(v, 16);
  return v + __shfl_xor(v, 32);
}

constexpr int RR_TR = 16;  // rows per wave
template <int T1, int T2, int T3>
__global__ __launch_bounds__(RR_WG, rr_occ<T1>()) void k_rows_reg(RowArgs A) {
  constexpr int CB = rr_cb<T1>();
  __shared__ float4 wl[2 * CB * 64];
  const int lane = threadIdx.x & 63, r = lane & 15, gq = lane >> 4;
  // workgroup pairs: even = the actor's pass over four row tiles, odd = the critic's over the same
  // tiles (the two nets share nothing but the tile's statistics slots, which they write apart)
  const int net = blockIdx.x & 1;
  const int tile = (blockIdx.x >> 1) * (RR_WG / 64) + (threadIdx.x >> 6);  // (B a multiple of 64: reg_shape)
  const int row0 = tile * RR_TR;
  const zbp_batch& bt = A.bt;
  const int NA = bt.num_actions;
  const float invB = 1.f / (float)bt.batch;
  const int64_t row = bt.idx[bt.idx_offset + row0 + r];
  float* ws = A.ws;
  float* st = ws + A.stats + (int64_t)tile * NSTAT;
  // the losses' inputs of this lane's row and actions (4 g + u, u < 4: num_actions <= 13 < 16), loaded
  // ahead of the forward passes so their latency hides under them
  const NetW& wa = A.n[0];
  const NetW& wc = A.n[1];
  RrStage<CB> wst;
  Tile z[2], dz[2];
  if (net == 0) {
  const float adv_in = bt.advantages[row], lp_in = bt.log_prob[row];
  float act_in[4], mu_in[4], sig_in[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    const int n = 4 * gq + u;
    act_in[u] = n < NA ? bt.actions[row * NA + n] : 0.f;
    mu_in[u] = n < NA ? bt.mu[row * NA + n] : 0.f;
    sig_in[u] = n < NA ? bt.sigma[row * NA + n] : 1.f;
  }

  // ---- actor: forward, Gaussian log-prob, clipped surrogate, KL; dL/dmu into dZ of the output
  // (every layer fetches the next layer's first weight chunk before its epilogue; the last forward
  // layer fetches the backward's)
  rr_fetch<2 * T1, CB>(ws + wa.wr[0], 0, wst);
  {
    Tile x0[2], x1[T1], x2[T2], x3[T3];
    rr_gather(wa, ws, row0, bt.obs, bt.obs_dim, row, x0);
    rr_forward<2, T1, false, true, T1 * T2, CB>(wa, 0, ws, wl, row0, x0, x1, wst, ws + wa.wr[1]);
    rr_forward<T1, T2, false, true, T2 * T3, CB>(wa, 1, ws, wl, row0, x1, x2, wst, ws + wa.wr[2]);
    rr_forward<T2, T3, false, true, T3 * 2, CB>(wa, 2, ws, wl, row0, x2, x3, wst, ws + wa.wr[3]);
    rr_forward<T3, 2, true, true, 2 * T3, CB>(wa, 3, ws, wl, row0, x3, z, wst, ws + wa.wtr[3]);
  }
  {
    // lane (r, g) holds actions 4 g + u (tile 0) and 16 + 4 g + u (tile 1) of row r
    const float kLog2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
    float lp = 0.f, kl = 0.f, diff[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = 16 * (j >> 2) + 4 * gq + (j & 3);
      diff[j] = 0.f;
      if (n < NA) {
        const float mu = z[j >> 2][j & 3], s = A.std_param[n];
        const float d = act_in[j & 3] - mu;  // (n < NA only in tile 0: j < 4)
        diff[j] = d;
        lp += -(d * d) / (2.f * (s * s)) - logf(s) - kLog2Pi;
        const float os = sig_in[j & 3], om = mu_in[j & 3];
        kl += logf(s / os + 1e-5f) + (os * os + (om - mu) * (om - mu)) / (2.f * (s * s)) - 0.5f;
      }
    }
    lp = rr_feat_sum(lp);
    kl = rr_feat_sum(kl);
    const float adv = adv_in, clip = A.lc.clip_param;
    const float ratio = expf(lp - lp_in);
    const float rc = fminf(fmaxf(ratio, 1.f - clip), 1.f + clip);
    const float s1 = -adv * ratio, s2 = -adv * rc;
    const float surr = fmaxf(s1, s2);
    // d max(s1, s2) / d ratio (torch.max splits a tie evenly; clamp passes the gradient inside
    // [1 - clip, 1 + clip], bounds included)
    const float in = (ratio >= 1.f - clip && ratio <= 1.f + clip) ? 1.f : 0.f;
    const float w1 = s1 > s2 ? 1.f : (s1 < s2 ? 0.f : 0.5f);
    const float g = (w1 * -adv + (1.f - w1) * -adv * in) * ratio * invB;  // dL / dlog_prob
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = 16 * (j >> 2) + 4 * gq + (j & 3);
      float d = 0.f, sg = 0.f;
      if (n < NA) {
        const float s = A.std_param[n];
        d = g * diff[j] / (s * s);
        sg = g * (diff[j] * diff[j] / (s * s * s) - 1.f / s);
      }
      dz[j >> 2][j & 3] = d;
      sg = rr_row_sum(sg);  // the std gradient summed over the tile's rows
      if (r == 0 && n < NA) st[3 + n] = sg;
    }
    rr_store_dz(wa, ws, row0, dz);
    const float su = wave_sum(gq == 0 ? surr : 0.f), ks = wave_sum(gq == 0 ? kl : 0.f);
    if (lane == 0) {
      st[0] = su;
      st[2] = ks;
      for (int a = 3 + NA; a < NSTAT; ++a) st[a] = 0.f;
    }
  }
  {
    Tile d3[T3], d2[T2], d1[T1];
    rr_backward<2, T3, T3 * T2, CB>(wa, 3, ws, wl, row0, dz, d3, wst, ws + wa.wtr[2]);
    rr_backward<T3, T2, T2 * T1, CB>(wa, 2, ws, wl, row0, d3, d2, wst, ws + wa.wtr[1]);
    rr_backward<T2, T1, 0, CB>(wa, 1, ws, wl, row0, d2, d1, wst, nullptr);
  }
  } else {
  const float tv_in = bt.values[row], ret_in = bt.returns[row];
  // ---- critic: forward, clipped value loss, backward
  rr_fetch<2 * T1, CB>(ws + wc.wr[0], 0, wst);
  {
    Tile x0[2], x1[T1], x2[T2], x3[T3];
    rr_gather(wc, ws, row0, bt.critic_obs, bt.critic_obs_dim, row, x0);
    rr_forward<2, T1, false, true, T1 * T2, CB>(wc, 0, ws, wl, row0, x0, x1, wst, ws + wc.wr[1]);
    rr_forward<T1, T2, false, true, T2 * T3, CB>(wc, 1, ws, wl, row0, x1, x2, wst, ws + wc.wr[2]);
    rr_forward<T2, T3, false, true, T3 * 2, CB>(wc, 2, ws, wl, row0, x2, x3, wst, ws + wc.wr[3]);
    rr_forward<T3, 2, true, true, 2 * T3, CB>(wc, 3, ws, wl, row0, x3, z, wst, ws + wc.wtr[3]);
  }
  {
    const float v = __shfl(z[0][0], r), tv = tv_in, ret = ret_in, clip = A.lc.clip_param;
    float vl, dv;
    if (A.lc.use_clipped_value_loss) {
      const float vd = v - tv;
      const float vc = tv + fminf(fmaxf(vd, -clip), clip);
      const float ea = (v - ret) * (v - ret), ec = (vc - ret) * (vc - ret);
      vl = fmaxf(ea, ec);
      const float wa_ = ea > ec ? 1.f : (ea < ec ? 0.f : 0.5f);
      const float in = (vd >= -clip && vd <= clip) ? 1.f : 0.f;
      dv = wa_ * 2.f * (v - ret) + (1.f - wa_) * 2.f * (vc - ret) * in;
    } else {
      vl = (ret - v) * (ret - v);
      dv = 2.f * (v - ret);
    }
    dv *= A.lc.value_loss_coef * invB;
#pragma unroll
    for (int j = 0; j < 8; ++j) dz[j >> 2][j & 3] = (gq == 0 && j == 0) ? dv : 0.f;
    rr_store_dz(wc, ws, row0, dz);
    const float vs = wave_sum(gq == 0 ? vl : 0.f);
    if (lane == 0) st[1] = vs;
  }
  {
    Tile d3[T3], d2[T2], d1[T1];
    rr_backward<2, T3, T3 * T2, CB>(wc, 3, ws, wl, row0, dz, d3, wst, ws + wc.wtr[2]);
    rr_backward<T3, T2, T2 * T1, CB>(wc, 2, ws, wl, row0, d3, d2, wst, ws + wc.wtr[1]);
    rr_backward<T2, T1, 0, CB>(wc, 1, ws, wl, row0, d2, d1, wst, nullptr);
  }
  }
}

// ------------------------------------------------------------------------------- k_wgrad
struct WgradArgs {
  NetW n[2];
  int tile0[2 * MAXL + 1], grp0[2 * MAXL + 1], blk0[2 * MAXL + 1], sp_nl[2 * MAXL], ord[2 * MAXL];
  int wtiles, ngroups, splits, batch;
  float* ws;
  int64_t part;
};
// dW_l = dZ_l^T X_l and db_l = sum dZ_l over the rows of one split. One workgroup = one block of up to
// 128 output rows (n) x 128 reduction columns (k) of one layer; its four waves take 64 x 64 quadrants
// (2 x 2 tiles of 32 x 32, v_mfma_f32_32x32x2_f32). The split's rows stream through LDS in chunks
// of 32 rows (four octets): dZ_l[n0 .. n0 + 127] and X_l[k0 .. k0 + 127] of a chunk are 2 x 4 contiguous
// 4 KB pieces of the octet-blocked row buffers (rbo), copied by all 256 threads into one of two
// buffers while the previous chunk is consumed (one barrier per chunk); every element is read from
// HBM / L2 once per block instead of once per wave. A wave reads its operands as float4 quads of
// rows (conflict-free ds_read_b128: a wave's 64 lanes cover one contiguous KB) and issues 16 MFMAs
// per octet. Partial tiles (and the bias column of the k0 = 0 tiles) go to the workspace in
// k_reduce's layout.
constexpr int WG_CHUNK_F = 2 * 4 * 128 * 8;  // floats of one chunk buffer (dZ + X: 32 KB)
__global__ __launch_bounds__(256, 2) void k_wgrad(WgradArgs A) {
  __shared__ float4 lds4[2 * WG_CHUNK_F / 4];
  float* lds = reinterpret_cast<float*>(lds4);
  // workgroup -> (net, layer) by the launch prefix, then (group, split) inside it, groups interleaved
  int pos = 0;
  while (pos + 1 < 2 * MAXL && A.blk0[pos + 1] <= (int)blockIdx.x) ++pos;
  const int nl = A.ord[pos];
  const int ng = A.grp0[nl + 1] - A.grp0[nl], local = (int)blockIdx.x - A.blk0[pos];
  const int grp = A.grp0[nl] + local % ng, split = local / ng, nsplit = A.sp_nl[nl];
  const NetW& w = A.n[nl / MAXL];
  const int l = nl % MAXL;
  const int P0 = w.p[l], P1 = w.p[l + 1], Tk = P0 / 32, Tn = P1 / 32, KG = (Tk + 3) / 4;
  const int t = threadIdx.x, wave = t >> 6, lane = t & 63, c = lane & 31, h = lane >> 5;
  const int g = grp - A.grp0[nl], nt0 = 4 * (g / KG), kt0 = 4 * (g % KG);
  const int nb = min(4, Tn - nt0), kb = min(4, Tk - kt0);  // tiles of the block
  const int C = A.batch / 32;  // the split's chunks [c0, c1)
  const int c0 = (int)((int64_t)split * C / nsplit), c1 = (int)((int64_t)(split + 1) * C / nsplit);
  const int r0 = 32 * c0, nch = c1 - c0;
  // chunk copy: per octet, dZ features n0 .. n0 + 32 nb - 1 and X features k0 .. k0 + 32 kb - 1 (8 rows each)
  const int fn = 32 * nb * 8 / 4, fk = 32 * kb * 8 / 4;  // float4s per octet
  const float4* gz = reinterpret_cast<const float4*>(A.ws + w.dz[l] + rbo(P1, 32 * nt0, r0));
  const float4* gx = reinterpret_cast<const float4*>(A.ws + w.x[l] + rbo(P0, 32 * kt0, r0));
  const int64_t oz = (int64_t)P1 * 2, ox = (int64_t)P0 * 2;  // float4 stride of an octet
  // thread t copies float4s t + 256 m, m < 8, of the chunk's 4 x 256 (dZ) + 4 x 256 (X) slots;
  // slot (part, octet o, float4 f = 2 feature + half) -> LDS float4 part 1024 + o 256 + half 128 + feature
  // (a wave's operand read, lane (c, h) at h 128 + feature c: every 16 lanes read 256 contiguous bytes)
  float4 st[8];
  auto fetch = [&](int ch) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int e = t + 256 * m, part = e >> 10, o = (e >> 8) & 3, f = e & 255;
      const int j = 4 * ch + o;  // octet of the split
      float4 v = float4{};
      if (part == 0) { if (f < fn) v = gz[j * oz + f]; }
      else if (f < fk) v = gx[j * ox + f];
      st[m] = v;
    }
  };
  auto stash = [&](int buf) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int e = t + 256 * m;
      lds4[buf * (WG_CHUNK_F / 4) + (e & ~255) + (e & 1) * 128 + ((e & 255) >> 1)] = st[m];
    }
  };
  // this wave's quadrant: n tiles 2 (wave >> 1) + {0, 1}, k tiles 2 (wave & 1) + {0, 1}
  const int qn = 2 * (wave >> 1), qk = 2 * (wave & 1);
  const bool on[2][2] = {{qn < nb && qk < kb, qn < nb && qk + 1 < kb}, {qn + 1 < nb && qk < kb, qn + 1 < nb && qk + 1 < kb}};
  const bool any = on[0][0];
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) acc[a][b] = f32x16{};
  float bsum[2] = {0.f, 0.f};
  const bool bias = kt0 == 0 && (wave & 1) == 0;
  fetch(0);
  stash(0);
  __syncthreads();
  if (nch > 1) fetch(1);
  for (int ch = 0; ch < nch; ++ch) {
    const float* bz = lds + (ch & 1) * WG_CHUNK_F;
    const float* bx = bz + 4096;
    if (any) {
#pragma unroll
      for (int o = 0; o < 4; ++o) {
        float4 za[2], xb[2];
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          za[a] = *reinterpret_cast<const float4*>(bz + o * 1024 + (h * 128 + 32 * (qn + a) + c) * 4);
          xb[a] = *reinterpret_cast<const float4*>(bx + o * 1024 + (h * 128 + 32 * (qk + a) + c) * 4);
        }
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] = mfma(za[a].x, xb[b].x, acc[a][b]);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] = mfma(za[a].y, xb[b].y, acc[a][b]);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] = mfma(za[a].z, xb[b].z, acc[a][b]);
#pragma unroll
        for (int a = 0; a < 2; ++a)
#pragma unroll
          for (int b = 0; b < 2; ++b) acc[a][b] = mfma(za[a].w, xb[b].w, acc[a][b]);
        if (bias)
#pragma unroll
          for (int a = 0; a < 2; ++a) bsum[a] += (za[a].x + za[a].y) + (za[a].z + za[a].w);
      }
    }
    if (ch + 1 < nch) stash((ch + 1) & 1);
    __syncthreads();  // chunk ch consumed by every wave, chunk ch + 1 in LDS
    if (ch + 2 < nch) fetch(ch + 2);
  }
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const float bs = bsum[a] + __shfl_xor(bsum[a], 32);
#pragma unroll
    for (int b = 0; b < 2; ++b)
      if (on[a][b]) {
        const int nt = nt0 + qn + a, kt = kt0 + qk + b;
        float* out = A.ws + A.part + ((int64_t)split * A.wtiles + A.tile0[nl] + nt * Tk + kt) * PART;
#pragma unroll
        for (int r = 0; r < 16; ++r) out[acc_row(r) * 32 + acc_col()] = acc[a][b][r];  // [n][k]
        if (kt == 0 && h == 0) out[1024 + c] = bs;
      }
  }
}

// ------------------------------------------------------------------------------- k_reduce
struct ReduceArgs {
  NetW n[2];
  int tile0[2 * MAXL + 1];
  int wtiles, splits, row_tiles, batch, num_actions;
  int sp_nl[2 * MAXL];
  float* gw[2][MAXL];
  float* gb[2][MAXL];
  const float* std_param;
  float* std_grad;
  float* stats;
  float entropy_coef;
  const float* ws;
  int64_t part, rstats;
  float* norm2;  // [wtiles + 1]: each tile's sum of squared gradients (the last: the std's), for zbp_optimizer_step
};
// one workgroup per weight tile: the split partials summed in order into .grad (weights of the tile,
// and the bias for k0 = 0) and the tile's sum of their squares (fixed order); the last workgroup: the
// scalars. 1024 threads: a thread sums one partial element over the splits with 16 loads in flight
// (with 256 threads and 8 in flight the launch waited on ~30 dependent rounds of partial loads)
constexpr int RED_THREADS = 1024;
__global__ __launch_bounds__(RED_THREADS) void k_reduce(ReduceArgs A) {
  if (blockIdx.x == (unsigned)A.wtiles) {
    // per-row-tile sums -> stats, the std gradient (+ the entropy bonus term): thread t < 256 sums row
    // tiles t, t + 256, ... (one row = 16 floats = four float4, two rows in flight), then a fixed-order
    // tree over those 256 (deterministic); the other threads only take part in the barriers
    __shared__ float red[256][NSTAT + 1];
    const int t = threadIdx.x;
    float sv[NSTAT];
#pragma unroll
    for (int q = 0; q < NSTAT; ++q) sv[q] = 0.f;
    const float4* rs = reinterpret_cast<const float4*>(A.ws + A.rstats);
    int rt = t < 256 ? t : A.row_tiles;
    for (; rt + 256 < A.row_tiles; rt += 512) {
      float4 v[8];
#pragma unroll
      for (int c = 0; c < 4; ++c) { v[c] = rs[(int64_t)rt * 4 + c]; v[4 + c] = rs[(int64_t)(rt + 256) * 4 + c]; }
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sv[4 * c] += v[c].x + v[4 + c].x; sv[4 * c + 1] += v[c].y + v[4 + c].y;
        sv[4 * c + 2] += v[c].z + v[4 + c].z; sv[4 * c + 3] += v[c].w + v[4 + c].w;
      }
    }
    for (; rt < A.row_tiles; rt += 256)
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float4 v = rs[(int64_t)rt * 4 + c];
        sv[4 * c] += v.x; sv[4 * c + 1] += v.y; sv[4 * c + 2] += v.z; sv[4 * c + 3] += v.w;
      }
    if (t < 256)
#pragma unroll
      for (int q = 0; q < NSTAT; ++q) red[t][q] = sv[q];
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
      if (t < st)
#pragma unroll
        for (int q = 0; q < NSTAT; ++q) red[t][q] += red[t + st][q];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      float tot[NSTAT];
      for (int q = 0; q < NSTAT; ++q) tot[q] = red[0][q];
      const float invB = 1.f / (float)A.batch;
      float ent = 0.f;
      for (int a = 0; a < A.num_actions; ++a) ent += 0.5f + 0.91893853320467274178f + logf(A.std_param[a]);
      A.stats[0] = tot[2] * invB;  // kl mean
      A.stats[1] = tot[1] * invB;  // value loss
      A.stats[2] = tot[0] * invB;  // surrogate loss
      A.stats[3] = ent;            // entropy (every row's)
      float ss = 0.f;
      for (int a = 0; a < A.num_actions; ++a) {
        const float g = tot[3 + a] - A.entropy_coef / A.std_param[a];
        A.std_grad[a] = g;
        ss += g * g;
      }
      A.norm2[A.wtiles] = ss;
    }
    return;
  }
  const int tile = blockIdx.x;
  int nl = 0;
  while (nl + 1 < 2 * MAXL && A.tile0[nl + 1] <= tile) ++nl;
  const int net = nl / MAXL, l = nl % MAXL;
  const NetW& w = A.n[net];
  const int t = tile - A.tile0[nl], kt = w.p[l] / 32;
  const int n0 = 32 * (t / kt), k0 = 32 * (t % kt);
  const int D0 = w.d[l], D1 = w.d[l + 1];
  float ss = 0.f;
  for (int e = threadIdx.x; e < PART; e += blockDim.x) {
    // (sixteen partial sums: sixteen split partials in flight per thread; a fixed order)
    float sv[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) sv[u] = 0.f;
    int sp = 0;
    const float* src = A.ws + A.part + (int64_t)tile * PART + e;
    const int64_t stride = (int64_t)A.wtiles * PART;
    const int nsp = A.sp_nl[nl];  // (this tile's layer's splits)
    for (; sp + 16 <= nsp; sp += 16)
#pragma unroll
      for (int u = 0; u < 16; ++u) sv[u] += src[(int64_t)(sp + u) * stride];
    for (; sp < nsp; ++sp) sv[0] += src[(int64_t)sp * stride];
    float s8[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) s8[u] = sv[u] + sv[u + 8];
    const float s = ((s8[0] + s8[1]) + (s8[2] + s8[3])) + ((s8[4] + s8[5]) + (s8[6] + s8[7]));
    if (e < 1024) {
      const int n = n0 + e / 32, k = k0 + e % 32;
      if (n < D1 && k < D0) { A.gw[net][l][(int64_t)n * D0 + k] = s; ss += s * s; }
    } else if (k0 == 0) {
      const int n = n0 + e - 1024;
      if (n < D1) { A.gb[net][l][n] = s; ss += s * s; }
    }
  }
  __shared__ float red[RED_THREADS / 64];
  ss = wave_sum(ss);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = ss;
  __syncthreads();
  if (threadIdx.x == 0) {
    float v = 0.f;
    for (int k = 0; k < RED_THREADS / 64; ++k) v += red[k];  // fixed order
    A.norm2[tile] = v;
  }
}

// ------------------------------------------------------------------------------- k_optim
struct OptimArgs {
  zbp_params P;
  float* lr;
  const float* stats;
  float* acc;
  float desired_kl, max_norm, b1, b2, eps;
  float* norm2;  // workspace scratch: nparts sums of squares (k_norm's per block or k_reduce's per tile), summed in order by k_adam
  int nparts;
  int64_t total;  // elements over all the tensors
};
// flat element g over the tensors in order -> (tensor t, element e): every thread's elements are
// independent loads (a loop over the tensors per thread would chain one memory round trip per tensor)
__device__ __forceinline__ void flat_elem(const zbp_params& P, int64_t g, int& t, int64_t& e) {
  t = 0;
  while (t + 1 < P.n_params && g >= P.numel[t]) { g -= P.numel[t]; ++t; }
  e = g;
}
__global__ __launch_bounds__(256) void k_norm(OptimArgs A) {
  // global gradient norm^2: per-block partial sums in a fixed order (deterministic)
  __shared__ float red[4];
  float s = 0.f;
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < A.total; f += (int64_t)gridDim.x * blockDim.x) {
    int t;
    int64_t e;
    flat_elem(A.P, f, t, e);
    const float g = A.P.grad[t][e];
    s += g * g;
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) A.norm2[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);  // fixed order
}
__global__ __launch_bounds__(256) void k_adam(OptimArgs A) {
  // learning rate rule (rsl_rl adaptive schedule, on the minibatch KL), clip coefficient, Adam
  const float lr = adaptive_lr(*A.lr, A.stats[0], A.desired_kl);
  // the global norm^2 from the partial sums: the first wave loads them lane-parallel and sums with a
  // butterfly (the same fixed order in every block), then shares it through LDS
  __shared__ float n2s;
  if (threadIdx.x < 64) {
    float v = 0.f;
    for (int b = threadIdx.x; b < A.nparts; b += 64) v += A.norm2[b];
    v = wave_sum(v);
    if (threadIdx.x == 0) n2s = v;
  }
  __syncthreads();
  const float total = sqrtf(n2s);
  const float coef = fminf(A.max_norm / (total + 1e-6f), 1.f);
  const float step = A.P.step[0][0] + 1.f;
  const float bc1 = 1.f - powf(A.b1, step), bc2s = sqrtf(1.f - powf(A.b2, step));
  const float step_size = lr / bc1;
  for (int64_t f = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; f < A.total; f += (int64_t)gridDim.x * blockDim.x) {
    int t;
    int64_t e;
    flat_elem(A.P, f, t, e);
    const float g = A.P.grad[t][e] * coef;
    A.P.grad[t][e] = g;
    const float m = A.b1 * A.P.exp_avg[t][e] + (1.f - A.b1) * g;
    const float v = A.b2 * A.P.exp_avg_sq[t][e] + (1.f - A.b2) * g * g;
    A.P.exp_avg[t][e] = m;
    A.P.exp_avg_sq[t][e] = v;
    A.P.param[t][e] -= step_size * m / (sqrtf(v) / bc2s + A.eps);
  }
  // (every block reads the old lr / step: the k_pack launch after this one writes the new ones)
}

// ------------------------------------------------------------------------------- rollout
// PPO.act (zbot_lab_amd/rl/ppo.py; rsl_rl ActorCritic.act + evaluate + get_actions_log_prob and
// RolloutStorage.add's transition fields) for one policy step of every env: one workgroup per 32
// rows gathers the observations (and writes them into the storage slot), runs the actor forward,
// draws a = mu + std * noise (noise = the caller's torch.randn_like), the Gaussian log-probability
// sum_a (-(a - mu)^2 / (2 std^2) - log std - log sqrt(2 pi)) and the critic's value; every
// transition field lands in the storage slot of this step, the actions also in `actions` (the
// env's input). The forward reads the workspace's weight images (zbp_pack).
struct ActArgs {
  NetW n[2];
  float* ws;
  const float* std_param;
  const float* obs;
  const float* cobs;
  const float* noise;   // the caller's draw, or nullptr: noise_at draws it
  const uint32_t* rng;  // (noise == nullptr) the workspace's draw counter
  int noise_step;
  uint32_t noise_seed;
  int obs_dim, cobs_dim, na, rows;
  float *actions, *s_obs, *s_cobs, *s_act, *s_val, *s_lp, *s_mu, *s_sig;
  int lds_x[MAXL], lds_out;
};
// The in-kernel action noise (zbp_act with io->noise == NULL): a standard normal per (row, action)
// from a counter-based draw -- splitmix64 of (the caller's seed, e.g. per rank; the workspace's draw
// counter, which every k_pack advances, so every rollout and every update; the rollout step; row;
// action), Box-Muller on its
// 24-bit halves. The same distribution as torch.randn, another stream; no launch of its own.
__device__ __forceinline__ uint64_t mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}
__device__ __forceinline__ float noise_at(const ActArgs& A, int row, int n) {
  if (A.noise) return A.noise[row * A.na + n];
  const uint64_t key = ((uint64_t)A.noise_seed << 32) ^ ((uint64_t)*A.rng << 12) ^ (uint64_t)(uint32_t)A.noise_step;
  const uint64_t h = mix64(mix64(key) ^ (uint64_t)((int64_t)row * A.na + n));
  const float u1 = ((float)(uint32_t)(h >> 40) + 1.f) * 5.9604644775390625e-8f;  // (0, 1]
  const float u2 = (float)(uint32_t)((h >> 16) & 0xFFFFFFu) * 5.9604644775390625e-8f;  // [0, 1)
  return sqrtf(-2.f * logf(u1)) * cosf(6.28318530717958647692f * u2);
}

__device__ void act_gather(const NetW& w, const float* src, int dim, float* st, int rows, float* lds, int lds_x0,
                           int row0) {
  const int P0 = w.p[0];
  for (int e = threadIdx.x; e < TR * P0; e += blockDim.x) {
    const int i = e / P0, k = e % P0;  // (row-major: the source rows are contiguous)
    const int row = row0 + i;
    const float v = (k < dim && row < rows) ? src[(int64_t)row * dim + k] : 0.f;
    lds[lds_x0 + i * (P0 + 4) + k] = v;
    if (k < dim && row < rows) st[(int64_t)row * dim + k] = v;
  }
  __syncthreads();
}
__global__ __launch_bounds__(256) void k_act(ActArgs A) {
  extern __shared__ float lds[];
  const int row0 = blockIdx.x * TR, tid = threadIdx.x;
  act_gather(A.n[0], A.obs, A.obs_dim, A.s_obs, A.rows, lds, A.lds_x[0], row0);
  net_forward_t<false>(A.n[0], A.ws, 0, A.lds_x, A.lds_out, lds, row0);
  if (tid < TR && row0 + tid < A.rows) {
    const int64_t row = row0 + tid;
    const float kLog2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
    float lp = 0.f;
    for (int a = 0; a < A.na; ++a) {
      const float mu = lds[A.lds_out + tid * 33 + a], s = A.std_param[a];
      const float x = mu + s * noise_at(A, row, a), diff = x - mu;
      lp += -(diff * diff) / (2.f * (s * s)) - logf(s) - kLog2Pi;
      A.actions[row * A.na + a] = x;
      A.s_act[row * A.na + a] = x;
      A.s_mu[row * A.na + a] = mu;
      A.s_sig[row * A.na + a] = s;
    }
    A.s_lp[row] = lp;
  }
  __syncthreads();  // (the output tile is reused by the critic)
  act_gather(A.n[1], A.cobs, A.cobs_dim, A.s_cobs, A.rows, lds, A.lds_x[0], row0);
  net_forward_t<false>(A.n[1], A.ws, 0, A.lds_x, A.lds_out, lds, row0);
  if (tid < TR && row0 + tid < A.rows) A.s_val[row0 + tid] = lds[A.lds_out + tid * 33];
}

// k_act on the register-resident forward (k_rows_reg's shapes): one wave per 16 rows, the weights
// shared through LDS
template <int T1, int T2, int T3>
#ifndef ZBP_ACT_REG_MIN
#define ZBP_ACT_REG_MIN 4096
#endif
#ifndef ZBP_ACT_SPLIT_MAX
#define ZBP_ACT_SPLIT_MAX 65536
#endif
__global__ __launch_bounds__(RR_WG, 2) void k_act_reg(ActArgs A) {
  constexpr int CB = 32;
  __shared__ float4 wl[2 * CB * 64];
  const int lane = threadIdx.x & 63, r = lane & 15, gq = lane >> 4;
  // workgroup pairs: even = the actor over four row tiles, odd = the critic over the same tiles
  const int net = blockIdx.x & 1;
  const int row0 = ((blockIdx.x >> 1) * (RR_WG / 64) + (threadIdx.x >> 6)) * RR_TR;  // (waves past the rows run on zeros, store nothing)
  const int64_t row = row0 + r;
  const bool ok = row < A.rows;
  const int na = A.na;
  Tile z[2];
  RrStage<CB> wst;
  rr_fetch<2 * T1, CB>(A.ws + A.n[net].wr[0], 0, wst);
  {
    const NetW& w = A.n[net];
    const int dim = net ? A.cobs_dim : A.obs_dim;
    const float* src = (net ? A.cobs : A.obs) + row * dim;
    float* st = (net ? A.s_cobs : A.s_obs) + row * dim;
    Tile x0[2], x1[T1], x2[T2], x3[T3];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * (j >> 2) + 4 * gq + (j & 3);
      const float v = (ok && k < dim) ? src[k] : 0.f;
      x0[j >> 2][j & 3] = v;
      if (ok && k < dim) st[k] = v;
    }
    rr_forward<2, T1, false, false, T1 * T2, CB>(w, 0, A.ws, wl, 0, x0, x1, wst, A.ws + w.wr[1]);
    rr_forward<T1, T2, false, false, T2 * T3, CB>(w, 1, A.ws, wl, 0, x1, x2, wst, A.ws + w.wr[2]);
    rr_forward<T2, T3, false, false, T3 * 2, CB>(w, 2, A.ws, wl, 0, x2, x3, wst, A.ws + w.wr[3]);
    rr_forward<T3, 2, true, false, 0, CB>(w, 3, A.ws, wl, 0, x3, z, wst, nullptr);
    if (net == 0) {
      // lane (r, g) holds actions 4 g + u and 16 + 4 g + u of row r
      const float kLog2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
      float lp = 0.f;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int n = 16 * (j >> 2) + 4 * gq + (j & 3);
        if (ok && n < na) {
          const float mu = z[j >> 2][j & 3], s = A.std_param[n];
          const float x = mu + s * noise_at(A, row, n), diff = x - mu;
          lp += -(diff * diff) / (2.f * (s * s)) - logf(s) - kLog2Pi;
          A.actions[row * na + n] = x;
          A.s_act[row * na + n] = x;
          A.s_mu[row * na + n] = mu;
          A.s_sig[row * na + n] = s;
        }
      }
      lp = rr_feat_sum(lp);
      if (ok && gq == 0) A.s_lp[row] = lp;
    } else if (ok && gq == 0) {
      A.s_val[row] = z[0][0];
    }
  }
}

// k_act for rollouts of the 128-wide nets (rsl_rl's [128, 128, 128], walking v2; round 6): one
// workgroup of four waves per 16-row tile and net, the waves splitting every layer's output tiles
// (a quarter each) and exchanging the layer's activations through LDS (double-buffered, one barrier
// per layer); each wave reads its own output tiles' weight blocks from L2 (no staging). At 4096 rows
// that is 2048 waves (two per SIMD) with a quarter of k_act_reg's MFMAs each, against k_act_reg's 512
// waves holding the whole net. Same statement (same per-lane accumulation order within a tile).
template <int TI, int TO, bool kElu>
__device__ __forceinline__ void as_layer(const float* __restrict__ img, const float* __restrict__ bias,
                                         const Tile (&in)[TI], Tile (&out)[TO], Tile* __restrict__ xs, int wv,
                                         int lane) {
  constexpr int TQ = TO / 4;
  const float4* g = reinterpret_cast<const float4*>(img);
  float4 wb[TI][TQ];
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int q = 0; q < TQ; ++q) wb[i][q] = g[(i * TO + wv * TQ + q) * 64 + lane];
  Tile acc[TQ];
#pragma unroll
  for (int q = 0; q < TQ; ++q) acc[q] = Tile{};
#pragma unroll
  for (int i = 0; i < TI; ++i)
#pragma unroll
    for (int q = 0; q < TQ; ++q) {
      Tile a = acc[q];
      a = mfma16(wb[i][q].x, in[i][0], a);
      a = mfma16(wb[i][q].y, in[i][1], a);
      a = mfma16(wb[i][q].z, in[i][2], a);
      a = mfma16(wb[i][q].w, in[i][3], a);
      acc[q] = a;
    }
  const float* bp = bias + 4 * ((lane & 63) >> 4);
#pragma unroll
  for (int q = 0; q < TQ; ++q) {
    const int o = wv * TQ + q;
    const float4 bq = *reinterpret_cast<const float4*>(bp + 16 * o);
    const float bv[4] = {bq.x, bq.y, bq.z, bq.w};
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      float v = acc[q][u] + bv[u];
      if (kElu) v = v > 0.f ? v : expf(v) - 1.f;  // ELU(alpha = 1), as ATen's elu kernel
      acc[q][u] = v;
    }
    xs[o * 64 + lane] = acc[q];
  }
  __syncthreads();
#pragma unroll
  for (int o = 0; o < TO; ++o) out[o] = xs[o * 64 + lane];
}

template <int T1, int T2, int T3>
__global__ __launch_bounds__(256, 2) void k_act_split(ActArgs A) {
  static_assert(T1 % 4 == 0 && T2 % 4 == 0 && T3 % 4 == 0, "output tiles split over four waves");
  constexpr int TM = T1 > T2 ? (T1 > T3 ? T1 : T3) : (T2 > T3 ? T2 : T3);
  __shared__ Tile xs[2][TM * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, r = lane & 15, gq = lane >> 4;
  const int net = blockIdx.x & 1;
  const int64_t row = (int64_t)(blockIdx.x >> 1) * 16 + r;
  const bool ok = row < A.rows;
  const int na = A.na;
  const NetW& w = A.n[net];
  Tile x0[2], x1[T1], x2[T2], x3[T3];
  {
    const int dim = net ? A.cobs_dim : A.obs_dim;
    const float* src = (net ? A.cobs : A.obs) + row * dim;
    float* st = (net ? A.s_cobs : A.s_obs) + row * dim;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int k = 16 * (j >> 2) + 4 * gq + (j & 3);
      const float v = (ok && k < dim) ? src[k] : 0.f;
      x0[j >> 2][j & 3] = v;
      if (wv == 0 && ok && k < dim) st[k] = v;
    }
  }
  as_layer<2, T1, true>(A.ws + w.wr[0], A.ws + w.bp[0], x0, x1, xs[0], wv, lane);
  as_layer<T1, T2, true>(A.ws + w.wr[1], A.ws + w.bp[1], x1, x2, xs[1], wv, lane);
  as_layer<T2, T3, true>(A.ws + w.wr[2], A.ws + w.bp[2], x2, x3, xs[0], wv, lane);
  if (wv != 0) return;
  // the output layer (2 tiles in the image: num_actions <= 13 and the value live in tile 0), wave 0
  Tile z = Tile{};
  {
    const float4* g = reinterpret_cast<const float4*>(A.ws + w.wr[3]);
#pragma unroll
    for (int i = 0; i < T3; ++i) {
      const float4 wq = g[(i * 2 + 0) * 64 + lane];
      z = mfma16(wq.x, x3[i][0], z);
      z = mfma16(wq.y, x3[i][1], z);
      z = mfma16(wq.z, x3[i][2], z);
      z = mfma16(wq.w, x3[i][3], z);
    }
    const float4 bq = *reinterpret_cast<const float4*>(A.ws + w.bp[3] + 4 * gq);
    z[0] += bq.x; z[1] += bq.y; z[2] += bq.z; z[3] += bq.w;
  }
  if (net == 0) {
    // lane (r, g) holds actions 4 g + u of row r
    const float kLog2Pi = 0.91893853320467274178f;  // log(sqrt(2 pi))
    float lp = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int n = 4 * gq + u;
      if (ok && n < na) {
        const float mu = z[u], s = A.std_param[n];
        const float x = mu + s * noise_at(A, row, n), diff = x - mu;
        lp += -(diff * diff) / (2.f * (s * s)) - logf(s) - kLog2Pi;
        A.actions[row * na + n] = x;
        A.s_act[row * na + n] = x;
        A.s_mu[row * na + n] = mu;
        A.s_sig[row * na + n] = s;
      }
    }
    lp = rr_feat_sum(lp);
    if (ok && gq == 0) A.s_lp[row] = lp;
  } else if (ok && gq == 0) {
    A.s_val[row] = z[0];
  }
}

// PPO.process_env_step + the runner's episode bookkeeping (zbot_lab_amd/rl/runner.py _rollout) for
// one step, one workgroup: the storage slot's reward (+ gamma * value on time-outs, rsl_rl's
// bootstrap) and done; cur_rew += reward, cur_len += 1; over the done envs ep_stats += {sum cur_rew,
// sum cur_len, count} (a fixed-order block reduction), then their cur_rew / cur_len are cleared.
__global__ __launch_bounds__(1024) void k_env_post(const float* __restrict__ rew, const int64_t* __restrict__ done,
                                                   const uint8_t* __restrict__ tout, const float* __restrict__ val,
                                                   float gamma, float* __restrict__ s_rew, float* __restrict__ s_done,
                                                   float* __restrict__ cur_rew, float* __restrict__ cur_len,
                                                   float* __restrict__ ep_stats, int n) {
  __shared__ float red[3][16];
  float a0 = 0.f, a1 = 0.f, a2 = 0.f;
  // four envs per thread in flight (the loads of all four issued before the first is used: one
  // memory round trip instead of four); the same envs in the same order per thread as one at a time
  constexpr int U = 4;
  for (int e0 = threadIdx.x; e0 < n; e0 += U * blockDim.x) {
    float r[U], v[U], cr0[U], cl0[U];
    int64_t dd[U];
    uint8_t to[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = min(e0 + u * (int)blockDim.x, n - 1);
      r[u] = rew[e];
      dd[u] = done[e];
      v[u] = val[e];
      to[u] = tout ? tout[e] : 0;
      cr0[u] = cur_rew[e];
      cl0[u] = cur_len[e];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int e = e0 + u * (int)blockDim.x;
      if (e < n) {
        const bool d = dd[u] > 0;
        float t = gamma * v[u];
        asm volatile("" : "+v"(t));  // (torch rounds the product, then the sum: no fma contraction)
        s_rew[e] = to[u] ? r[u] + t : r[u];
        s_done[e] = (float)dd[u];
        const float cr = cr0[u] + r[u], cl = cl0[u] + 1.f;
        if (d) { a0 += cr; a1 += cl; a2 += 1.f; }
        cur_rew[e] = d ? 0.f : cr;
        cur_len[e] = d ? 0.f : cl;
      }
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    a0 += __shfl_xor(a0, o);
    a1 += __shfl_xor(a1, o);
    a2 += __shfl_xor(a2, o);
  }
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = a0;
    red[1][threadIdx.x >> 6] = a1;
    red[2][threadIdx.x >> 6] = a2;
  }
  __syncthreads();
  if (threadIdx.x < 3) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[threadIdx.x][w];
    ep_stats[threadIdx.x] += t;
  }
}

// ------------------------------------------------------------------------------- GAE
// RolloutStorage.compute_returns (zbot_lab_amd/rl/ppo.py; rsl_rl GAE with time-out bootstrapping
// already folded into the rewards): one thread per env runs the backward recursion over T steps;
// advantages = returns - values, then normalised by the mean and the unbiased std over all T x N.
// Partial sums per block in a fixed order (deterministic).
constexpr int GAE_BLOCKS = 256;
__global__ __launch_bounds__(256) void k_gae(const float* __restrict__ rew, const float* __restrict__ done,
                                             const float* __restrict__ val, const float* __restrict__ last,
                                             float* __restrict__ ret, float* __restrict__ adv, int T, int N, float gamma,
                                             float lam, float* __restrict__ part) {
  __shared__ float red[4];
  float s = 0.f;
  for (int n = blockIdx.x * blockDim.x + threadIdx.x; n < N; n += gridDim.x * blockDim.x) {
    float a = 0.f, next = last[n];
    for (int k = T - 1; k >= 0; --k) {
      const int64_t e = (int64_t)k * N + n;
      const float v = val[e], nt = 1.f - done[e];
      // torch rounds every product and sum of the recursion (one kernel per op): no fma contraction
      float p = nt * gamma * next, q = nt * gamma * lam * a;
      asm volatile("" : "+v"(p), "+v"(q));
      const float delta = rew[e] + p - v;
      a = delta + q;
      const float r = a + v;
      ret[e] = r;
      const float d = r - v;
      adv[e] = d;
      s += d;
      next = v;
    }
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}
// one block: the mean, then the unbiased variance around it -> part[GAE_BLOCKS .. +2] = {mean, std + 1e-8}
__global__ __launch_bounds__(1024) void k_adv_stats(const float* __restrict__ adv, int64_t M, float* __restrict__ part) {
  __shared__ float red[16];
  __shared__ float mean_s;
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int b = 0; b < GAE_BLOCKS; ++b) t += part[b];
    mean_s = t / (float)M;
  }
  __syncthreads();
  const float mean = mean_s;
  float q = 0.f;
  for (int64_t e = threadIdx.x; e < M; e += blockDim.x) {
    const float d = adv[e] - mean;
    q += d * d;
  }
  for (int o = 32; o > 0; o >>= 1) q += __shfl_xor(q, o);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
    part[GAE_BLOCKS] = mean;
    part[GAE_BLOCKS + 1] = sqrtf(t / (float)(M - 1)) + 1e-8f;
  }
}
__global__ __launch_bounds__(256) void k_adv_norm(float* __restrict__ adv, int64_t M, const float* __restrict__ part) {
  const float mean = part[GAE_BLOCKS], den = part[GAE_BLOCKS + 1];
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < M; e += (int64_t)gridDim.x * blockDim.x)
    adv[e] = (adv[e] - mean) / den;  // (a division, as torch's (adv - mean) / (std + 1e-8))
}

// k_rows_reg instantiation for the nets' shape: 1 = hidden [256, 256, 128], 2 = [128, 128, 128] (both
// nets; inputs / outputs <= 32), 0 = none (k_rows)
int reg_shape(const Layout& lo, int B = 128) {
  if (B % 64) return 0;  // (k_rows_reg: whole workgroups of four 16-row tiles)
  const char* e = getenv("ZBP_ROWS");  // (read per call: tests switch it)
  if (e && strcmp(e, "lds") == 0) return 0;
  const NetW &a = lo.n[0], &c = lo.n[1];
  if (a.L != 4 || c.L != 4) return 0;
  for (int l = 0; l <= 4; ++l)
    if (a.p[l] != c.p[l]) return 0;
  if (a.p[0] != 32 || a.p[4] != 32) return 0;
  if (a.p[1] == 256 && a.p[2] == 256 && a.p[3] == 128) return 1;
  if (a.p[1] == 128 && a.p[2] == 128 && a.p[3] == 128) return 2;
  return 0;
}

int launch_check(const char* what) {
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? 0 : hip_fail(e, what);
}

PackArgs pack_args(const Layout& lo, const zbp_net* a, const zbp_net* c, float* ws) {
  PackArgs P{};
  P.n[0] = lo.n[0];
  P.n[1] = lo.n[1];
  const zbp_net* nets[2] = {a, c};
  for (int k = 0; k < 2; ++k)
    for (int l = 0; l < nets[k]->n_layers; ++l) { P.w[k][l] = nets[k]->w[l]; P.b[k][l] = nets[k]->b[l]; }
  P.ws = ws;
  P.rng = reinterpret_cast<uint32_t*>(ws + lo.rng);
  return P;
}
int do_pack(const Layout& lo, const zbp_net* a, const zbp_net* c, float* ws, hipStream_t s,
            const PackArgs* tail = nullptr) {
  const int L = lo.n[0].L > lo.n[1].L ? lo.n[0].L : lo.n[1].L;
  PackArgs P = pack_args(lo, a, c, ws);
  if (tail) {
    P.tail = 1;
    P.n_params = tail->n_params;
    P.lr = tail->lr;
    P.stats = tail->stats;
    P.acc = tail->acc;
    P.desired_kl = tail->desired_kl;
    for (int t = 0; t < tail->n_params; ++t) P.step[t] = tail->step[t];
  }
  k_pack<<<dim3(64, 2, L), 256, 0, s>>>(P);
  return launch_check("k_pack");
}

}  // namespace

extern "C" {

const char* zbp_last_error(void) { return g_err; }

int64_t zbp_workspace_floats(const zbp_net* actor, const zbp_net* critic, int32_t batch) {
  if (check_net(actor) || check_net(critic) || batch < TR || batch % TR) return -1;
  return make_layout(actor, critic, batch).total;
}

int zbp_pack(const zbp_net* actor, const zbp_net* critic, float* ws, int32_t batch, void* stream) {
  if (const char* e = check_net(actor)) return fail(-1, e);
  if (const char* e = check_net(critic)) return fail(-1, e);
  if (!ws || batch < TR || batch % TR) return fail(-1, "zbp_pack: workspace / batch");
  return do_pack(make_layout(actor, critic, batch), actor, critic, ws, (hipStream_t)stream);
}

int zbp_minibatch(const zbp_net* actor, const zbp_net* critic, const float* std_param, float* std_grad,
                  const zbp_batch* batch, const zbp_loss_cfg* loss, float* ws, float* stats, void* stream) {
  if (const char* e = check_net(actor)) return fail(-1, e);
  if (const char* e = check_net(critic)) return fail(-1, e);
  if (!batch || !loss || !ws || !stats || !std_param || !std_grad) return fail(-1, "zbp_minibatch: null argument");
  const int B = batch->batch;
  if (B < TR || B % TR) return fail(-1, "zbp_minibatch: batch must be a positive multiple of 32");
  if (batch->num_actions != actor->dim[actor->n_layers] || batch->num_actions > NSTAT - 3)
    return fail(-1, "zbp_minibatch: num_actions must match the actor output (<= 13)");
  if (batch->obs_dim != actor->dim[0] || batch->critic_obs_dim != critic->dim[0] || critic->dim[critic->n_layers] != 1)
    return fail(-1, "zbp_minibatch: observation dims / critic output");
  for (int k = 0; k < 2; ++k) {
    const zbp_net* n = k ? critic : actor;
    for (int l = 0; l < n->n_layers; ++l)
      if (!n->gw[l] || !n->gb[l]) return fail(-1, "zbp_minibatch: null .grad buffer");
  }
  hipStream_t s = (hipStream_t)stream;
  const Layout lo = make_layout(actor, critic, B);

  RowArgs R{};
  R.n[0] = lo.n[0];
  R.n[1] = lo.n[1];
  R.bt = *batch;
  R.lc = *loss;
  R.std_param = std_param;
  R.ws = ws;
  R.stats = lo.stats;
  R.B = B;
  int off = 0;
  for (int l = 0; l < MAXL; ++l) {
    const int p = lo.n[0].p[l] > lo.n[1].p[l] ? lo.n[0].p[l] : lo.n[1].p[l];
    R.lds_x[l] = off;
    off += TR * (p + 4);
  }
  R.lds_dz = off;  // the output layer's dZ ([32][p(L) + 4], p(L) = 32)
  off += TR * (32 + 4);
  R.lds_out = off;
  off += TR * 33;
  R.lds_red = off;
  off += NSTAT;
  const size_t lds = sizeof(float) * off;
  if (lds > 160 * 1024) return fail(-1, "zbp_minibatch: nets too wide for the LDS row tile");
  static bool lds_set = false;  // (a host-side attribute: set once, outside any stream capture's ops)
  if (!lds_set) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_rows, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute k_rows");
    lds_set = true;
  }
  // the register-resident row kernel for the shipped shapes (ZBP_ROWS=lds: the LDS one, for A/Bs)
  const int shape = reg_shape(lo, B);
  if (shape == 1)
    k_rows_reg<16, 16, 8><<<2 * (B / 64), RR_WG, 0, s>>>(R);
  else if (shape == 2)
    k_rows_reg<8, 8, 8><<<2 * (B / 64), RR_WG, 0, s>>>(R);
  else
    k_rows<<<B / TR, ROW_THREADS, lds, s>>>(R);
  if (int rc = launch_check("k_rows")) return rc;

  WgradArgs W{};
  W.n[0] = lo.n[0];
  W.n[1] = lo.n[1];
  for (int i = 0; i <= 2 * MAXL; ++i) W.tile0[i] = lo.tile0[i];
  for (int i = 0; i <= 2 * MAXL; ++i) W.grp0[i] = lo.grp0[i];
  for (int i = 0; i <= 2 * MAXL; ++i) W.blk0[i] = lo.blk0[i];
  for (int i = 0; i < 2 * MAXL; ++i) W.sp_nl[i] = lo.sp_nl[i];
  for (int i = 0; i < 2 * MAXL; ++i) W.ord[i] = lo.ord[i];
  W.wtiles = lo.wtiles;
  W.ngroups = lo.ngroups;
  W.splits = lo.splits;
  W.batch = B;
  W.ws = ws;
  W.part = lo.part;
  k_wgrad<<<lo.blk0[2 * MAXL], 256, 0, s>>>(W);
  if (int rc = launch_check("k_wgrad")) return rc;

  ReduceArgs D{};
  D.n[0] = lo.n[0];
  D.n[1] = lo.n[1];
  for (int i = 0; i <= 2 * MAXL; ++i) D.tile0[i] = lo.tile0[i];
  D.wtiles = lo.wtiles;
  D.splits = lo.splits;
  for (int i = 0; i < 2 * MAXL; ++i) D.sp_nl[i] = lo.sp_nl[i];
  D.row_tiles = shape ? B / RR_TR : B / TR;
  D.batch = B;
  D.num_actions = batch->num_actions;
  for (int k = 0; k < 2; ++k) {
    const zbp_net* n = k ? critic : actor;
    for (int l = 0; l < n->n_layers; ++l) {
      D.gw[k][l] = n->gw[l];
      D.gb[k][l] = n->gb[l];
    }
  }
  D.std_param = std_param;
  D.std_grad = std_grad;
  D.stats = stats;
  D.entropy_coef = loss->entropy_coef;
  D.ws = ws;
  D.part = lo.part;
  D.rstats = lo.stats;
  D.norm2 = ws + lo.scratch;
  k_reduce<<<lo.wtiles + 1, RED_THREADS, 0, s>>>(D);
  return launch_check("k_reduce");
}

int zbp_optimizer_step(const zbp_params* params, float* lr, const float* stats, float* acc, float desired_kl,
                       float max_grad_norm, float beta1, float beta2, float eps, const zbp_net* actor,
                       const zbp_net* critic, float* ws, int32_t batch, int32_t norm_from_minibatch, void* stream) {
  if (!params || params->n_params < 1 || params->n_params > ZBP_MAX_PARAMS || !lr || !stats || !acc || !ws)
    return fail(-1, "zbp_optimizer_step: bad argument");
  if (const char* e = check_net(actor)) return fail(-1, e);
  if (const char* e = check_net(critic)) return fail(-1, e);
  hipStream_t s = (hipStream_t)stream;
  const Layout lo = make_layout(actor, critic, batch);
  OptimArgs O{};
  O.P = *params;
  O.lr = lr;
  O.stats = stats;
  O.acc = acc;
  O.desired_kl = desired_kl;
  O.max_norm = max_grad_norm;
  O.b1 = beta1;
  O.b2 = beta2;
  O.eps = eps;
  O.norm2 = ws + lo.scratch;
  O.total = 0;
  for (int t = 0; t < params->n_params; ++t) O.total += params->numel[t];
  if (norm_from_minibatch) {
    O.nparts = lo.wtiles + 1;  // k_reduce's per-tile sums of the gradients it wrote
  } else {
    O.nparts = 64;
    k_norm<<<64, 256, 0, s>>>(O);
    if (int rc = launch_check("k_norm")) return rc;
  }
  k_adam<<<256, 256, 0, s>>>(O);
  if (int rc = launch_check("k_adam")) return rc;
  PackArgs T{};
  T.n_params = params->n_params;
  T.lr = lr;
  T.stats = stats;
  T.acc = acc;
  T.desired_kl = desired_kl;
  for (int t = 0; t < params->n_params; ++t) T.step[t] = params->step[t];
  return do_pack(lo, actor, critic, ws, s, &T);
}

int zbp_act(const zbp_net* actor, const zbp_net* critic, const float* std_param, const zbp_act_io* io, float* ws,
            int32_t batch, void* stream) {
  if (const char* e = check_net(actor)) return fail(-1, e);
  if (const char* e = check_net(critic)) return fail(-1, e);
  if (!io || !ws || !std_param || !io->obs || !io->critic_obs || !io->actions || !io->st_obs ||
      !io->st_critic_obs || !io->st_actions || !io->st_values || !io->st_log_prob || !io->st_mu || !io->st_sigma)
    return fail(-1, "zbp_act: null argument");
  if (io->rows < 1 || batch < TR || batch % TR) return fail(-1, "zbp_act: rows / batch");
  if (io->num_actions != actor->dim[actor->n_layers] || io->obs_dim != actor->dim[0] ||
      io->critic_obs_dim != critic->dim[0] || critic->dim[critic->n_layers] != 1)
    return fail(-1, "zbp_act: observation / action dims");
  const Layout lo = make_layout(actor, critic, batch);
  ActArgs A{};
  A.n[0] = lo.n[0];
  A.n[1] = lo.n[1];
  A.ws = ws;
  A.std_param = std_param;
  A.obs = io->obs;
  A.cobs = io->critic_obs;
  A.noise = io->noise;
  A.rng = reinterpret_cast<const uint32_t*>(ws + lo.rng);
  A.noise_step = io->noise_step;
  A.noise_seed = (uint32_t)io->noise_seed;
  A.obs_dim = io->obs_dim;
  A.cobs_dim = io->critic_obs_dim;
  A.na = io->num_actions;
  A.rows = io->rows;
  A.actions = io->actions;
  A.s_obs = io->st_obs;
  A.s_cobs = io->st_critic_obs;
  A.s_act = io->st_actions;
  A.s_val = io->st_values;
  A.s_lp = io->st_log_prob;
  A.s_mu = io->st_mu;
  A.s_sig = io->st_sigma;
  int off = 0;
  for (int l = 0; l < MAXL; ++l) {
    const int p = lo.n[0].p[l] > lo.n[1].p[l] ? lo.n[0].p[l] : lo.n[1].p[l];
    A.lds_x[l] = off;
    off += TR * (p + 4);
  }
  A.lds_out = off;
  off += TR * 33;
  const size_t lds = sizeof(float) * off;
  if (lds > 160 * 1024) return fail(-1, "zbp_act: nets too wide for the LDS row tile");
  static bool lds_set = false;
  if (!lds_set) {
    const hipError_t e = hipFuncSetAttribute((const void*)k_act, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    if (e != hipSuccess) return hip_fail(e, "hipFuncSetAttribute k_act");
    lds_set = true;
  }
  // (the register-resident forward, actor and critic in separate workgroups, from ZBP_ACT_REG_MIN rows
  // (4096): 23.5 us against the LDS kernel's 34.9 at 4096 rows (before the split 42 us: too few
  // workgroups), 146 against 242 at 32 768 (profiles/r5y); ZBP_ACT=lds / reg for A/Bs)
  const char* ea = getenv("ZBP_ACT");
  const bool f_reg = ea && !strcmp(ea, "reg"), f_lds = ea && !strcmp(ea, "lds"), f_split = ea && !strcmp(ea, "split");
  const int reg_min = (f_reg || f_split) ? 0 : (f_lds ? (1 << 30) : ZBP_ACT_REG_MIN);
  const int shape = io->rows >= reg_min ? reg_shape(lo) : 0, wgs = 2 * ((io->rows + 63) / 64);
  // the 128-wide nets (shape 2): the split-output forward (k_act_split, round 6) up to
  // ZBP_ACT_SPLIT_MAX rows; ZBP_ACT=reg / lds / split forces a kernel for A/Bs and tests
  const bool split = shape == 2 && !f_reg && (f_split || io->rows <= ZBP_ACT_SPLIT_MAX);
  if (split)
    k_act_split<8, 8, 8><<<2 * ((io->rows + 15) / 16), 256, 0, (hipStream_t)stream>>>(A);
  else if (shape == 1)
    k_act_reg<16, 16, 8><<<wgs, RR_WG, 0, (hipStream_t)stream>>>(A);
  else if (shape == 2)
    k_act_reg<8, 8, 8><<<wgs, RR_WG, 0, (hipStream_t)stream>>>(A);
  else
    k_act<<<(io->rows + TR - 1) / TR, 256, lds, (hipStream_t)stream>>>(A);
  return launch_check("k_act");
}

int zbp_env_post(const float* rewards, const int64_t* dones, const uint8_t* time_outs, const float* values, float gamma,
                 float* st_rewards, float* st_dones, float* cur_rew, float* cur_len, float* ep_stats, int32_t n,
                 void* stream) {
  if (!rewards || !dones || !values || !st_rewards || !st_dones || !cur_rew || !cur_len || !ep_stats || n < 1)
    return fail(-1, "zbp_env_post: bad argument");
  k_env_post<<<1, 1024, 0, (hipStream_t)stream>>>(rewards, dones, time_outs, values, gamma, st_rewards, st_dones, cur_rew,
                                                  cur_len, ep_stats, n);
  return launch_check("k_env_post");
}

int zbp_gae(const float* rewards, const float* dones, const float* values, const float* last_values, float* returns,
            float* advantages, int32_t steps, int32_t envs, float gamma, float lam, int32_t normalize, float* scratch,
            void* stream) {
  if (!rewards || !dones || !values || !last_values || !returns || !advantages || !scratch || steps < 1 || envs < 1)
    return fail(-1, "zbp_gae: bad argument");
  hipStream_t s = (hipStream_t)stream;
  k_gae<<<GAE_BLOCKS, 256, 0, s>>>(rewards, dones, values, last_values, returns, advantages, steps, envs, gamma, lam,
                                   scratch);
  if (int rc = launch_check("k_gae")) return rc;
  if (!normalize) return 0;
  const int64_t M = (int64_t)steps * envs;
  k_adv_stats<<<1, 1024, 0, s>>>(advantages, M, scratch);
  if (int rc = launch_check("k_adv_stats")) return rc;
  k_adv_norm<<<256, 256, 0, s>>>(advantages, M, scratch);
  return launch_check("k_adv_norm");
}

}  // extern "C"
