// zbot_sim.hip — MI355X (gfx950) batched ZBOT-6 simulator: one fused kernel per policy step.
//
// Replaces, for zbot-6b-walking-v2, the reference's DirectRLEnv.step:
//   _pre_physics_step (v2.py:276-287) -> 4 x [ImplicitActuator + PhysX articulation/contact
//   substep] -> ContactSensor update -> _get_dones (v2.py:384-411) -> _get_rewards
//   (v2.py:371-382, terms 461-561) -> _reset_idx (v2.py:413-459) -> _get_observations
//   (v2.py:312-369)      [v2.py = source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6dof_bipedal_env_v2.py]
//
// Mapping: one env per 16-lane team (one DPP row), 4 envs per 64-lane wave =
// workgroup, N/4 workgroups renumbered XCD-major. Persistent state is SoA [field][env] in HBM,
// read once and written once per step; lane s of a team loads / stores rows s + 16k, so one
// instruction moves 16 rows x 4 envs. Model constants are wave-uniform (scalar loads). Within a
// team: FK as a DPP prefix over the chain, RNEA / CRBA one body per lane, the 12x12 Cholesky with
// one row per lane, ground contact one link per lane, self collision as a capsule broadphase +
// separating-axis test dealt over the lanes and GJK on DPP quads, PGS with lane s owning one
// whitened coordinate (row dots reduced by DPP). The contact rows (up to ZB_MAX_CONTACTS slots x 3
// directions x 12 coordinates) and the per-substep sensor records are staged in LDS. No MFMA: the
// largest dense contraction is 12x12 per env.
//
// The algorithm is the one restated on the CPU in oracle/zbot_oracle.c (the parity oracle);
// the two are written independently and compared by tests/test_gpu_parity.py.
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include "zbot.h"

namespace {

constexpr int NB = ZB_NUM_BODIES;
constexpr int ND = ZB_NUM_DOF;
constexpr int NL = ZB_NUM_LINKS;
constexpr int NV = 6 + ND;
constexpr int NCM = ZB_MAX_CONTACTS;
constexpr int NSELF = 18;  // self-collision candidates per env (canonical pair order), see the candidate list
constexpr int WAVE = 64;
constexpr float PI_F = 3.14159265358979323846f;
constexpr float TWO_PI_F = 6.28318530717958647692f;
constexpr float RIM_EPS = 1e-3f;  // m; 2% of the module radius (see detect)
// Self collision on the link shape written as a core hull + a ball of radius kCoreM (PhysX PCM
// style): the core is the hull of the two circles moved kCoreM into the shape along their normals
// with radius r - kCoreM; caps exact, rims rounded (= oracle CORE_M)
constexpr float kCoreM = 0.004f;
#ifndef ZB_GJK_MAXIT
#define ZB_GJK_MAXIT 16
#endif
constexpr int kGjkMaxIt = ZB_GJK_MAXIT;
#ifndef ZB_RSQ_NR
#define ZB_RSQ_NR 0
#endif
#ifndef ZB_GJK_TOL
#define ZB_GJK_TOL 1e-5f  // (variant builds for the A/B: scripts/gpu_r5_bench_ab.sh)
#endif
constexpr float kGjkTol = ZB_GJK_TOL;  // m: GJK stops when its distance bounds are this close
constexpr float kGjkTilt = 0.01f;  // warm start: tilt of the first three support directions (rad)

// The ZBOT-6 chain topology is compiled in (zb_create checks the model against it):
// link l belongs to composite body (l+1)/2; joint j connects body j -> j+1.
__host__ __device__ constexpr int link_body(int l) { return (l + 1) >> 1; }

// Model pointer in the constant address space (4): wave-uniform loads through it are scalar
// (s_load) and land in SGPRs, never in per-lane VGPRs.
using MP = const __attribute__((address_space(4))) zb_model*;
using CF = const __attribute__((address_space(4))) float;
template <int N>
__device__ __forceinline__ void ldc(float (&d)[N], CF* s) {
#pragma unroll
  for (int i = 0; i < N; ++i) d[i] = s[i];
}
__device__ __forceinline__ MP to_mp(const zb_model* m) { return (MP)(uintptr_t)m; }

// ------------------------------------------------------------------------- diagnostic stamps
// Built only with -DZB_STAMPS (python -m zbot_lab_amd.build --stamps): s_memtime deltas per phase,
// summed per wave (lane 0) into g_stamps. Never part of the measured product build.
constexpr int NSTAMP = 16;
constexpr int kStampCount0 = 13;  // slots 13, 14 count events (GJK calls, iterations); 15 = max wave cycles
constexpr int kStampSub = 8;      // substep end times per wave record (>= MAXSUB)
#ifdef ZB_STAMPS
__device__ unsigned long long g_stamps[NSTAMP];
__device__ unsigned long long g_stamp_slowest[NSTAMP];  // phase cycles of the slowest wave seen
// per-launch wave histograms: [0, 64) the wave's largest number of GJK pairs of one env in one
// substep; [64, 128) the wave's largest per-lane sum of GJK iterations over the step, in bins of 4;
// contact-cap counters over env-substeps: [128] env-substeps, [129] more than NCM candidates (the
// cap selects), [130] more than NSELF self contacts, [131] self contacts on overlapping cores (the
// centre-difference fallback), [132] env-substeps with such a contact, [133] self contacts,
// [134] ground candidates
constexpr int kCapCounters = 128;
__device__ unsigned long long g_stamp_hist[kCapCounters + 8];
// per-workgroup record of the latest launch (zb_read_wave_times): start / end on the constant-rate
// clock (s_memrealtime, 100 MHz, comparable across CUs) and the wave's phase cycles
constexpr int kWaveRec = 2 + kStampCount0 + kStampSub, kMaxWaveRecs = 1 << 16;
__device__ unsigned long long g_wave_rec[kMaxWaveRecs][kWaveRec];
struct Stamps {
  unsigned long long t, rt0, rsub[kStampSub], acc[NSTAMP];
  unsigned umax, itsum;
  __device__ void begin() {
    rt0 = __builtin_amdgcn_s_memrealtime();
    for (int k = 0; k < kStampSub; ++k) rsub[k] = 0;
    t = __builtin_amdgcn_s_memtime();
    for (int k = 0; k < NSTAMP; ++k) acc[k] = 0;
    umax = 0; itsum = 0;
  }
  __device__ void note_pairs(unsigned u) { umax = u > umax ? u : umax; }
  // contact-cap counters of one env-substep (called by the team lead)
  __device__ void note_caps(int n_ground, int n_self, int n_deep) {
#ifdef ZB_STAMPS_NO_CAPS  // (timing runs: the counters' global atomics would skew the phases)
    return;
#endif
    atomicAdd(&g_stamp_hist[kCapCounters], 1ull);
    if (n_ground + min(n_self, NSELF) > NCM) atomicAdd(&g_stamp_hist[kCapCounters + 1], 1ull);
    if (n_self > NSELF) atomicAdd(&g_stamp_hist[kCapCounters + 2], 1ull);
    if (n_deep) {
      atomicAdd(&g_stamp_hist[kCapCounters + 3], (unsigned long long)n_deep);
      atomicAdd(&g_stamp_hist[kCapCounters + 4], 1ull);
    }
    if (n_self) atomicAdd(&g_stamp_hist[kCapCounters + 5], (unsigned long long)n_self);
    if (n_ground) atomicAdd(&g_stamp_hist[kCapCounters + 6], (unsigned long long)n_ground);
  }
  __device__ void note_its(unsigned its) { itsum += its; }
  __device__ void substep_end(int k) { rsub[k] = __builtin_amdgcn_s_memrealtime(); }
  __device__ void mark(int k) {
    const unsigned long long n = __builtin_amdgcn_s_memtime();
    acc[k] += n - t;
    t = n;
  }
  // per-lane event counts (slots >= kStampCount0), summed over every lane at flush
  __device__ void count(int k, unsigned v) { acc[k] += v; }
  __device__ void flush() {
    if ((threadIdx.x & 63) == 0 && blockIdx.x < kMaxWaveRecs) {
      g_wave_rec[blockIdx.x][0] = rt0;
      g_wave_rec[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
      for (int k = 0; k < kStampCount0; ++k) g_wave_rec[blockIdx.x][2 + k] = acc[k];
      for (int k = 0; k < kStampSub; ++k) g_wave_rec[blockIdx.x][2 + kStampCount0 + k] = rsub[k];
    }
#ifdef ZB_STAMPS_WAVE_ONLY  // timing runs: no contended global atomics while other waves still run
    return;
#endif
    if ((threadIdx.x & 63) == 0)
      for (int k = 0; k < kStampCount0; ++k) atomicAdd(&g_stamps[k], acc[k]);
    for (int k = kStampCount0; k < NSTAMP - 1; ++k)
      if (acc[k]) atomicAdd(&g_stamps[k], acc[k]);
    unsigned um = umax, im = itsum;
    for (int o = 32; o > 0; o >>= 1) {
      const unsigned a = __shfl_xor(um, o), b = __shfl_xor(im, o);
      um = a > um ? a : um;
      im = b > im ? b : im;
    }
    if ((threadIdx.x & 63) == 0) {
      atomicAdd(&g_stamp_hist[um < 63 ? um : 63], 1ull);
      atomicAdd(&g_stamp_hist[64 + (im / 4 < 63 ? im / 4 : 63)], 1ull);
    }
    if ((threadIdx.x & 63) == 0) {  // slot NSTAMP - 1: the slowest wave's cycles over the launches
      unsigned long long tot = 0;
      for (int k = 0; k < kStampCount0; ++k) tot += acc[k];
      const unsigned long long old = atomicMax(&g_stamps[NSTAMP - 1], tot);
      if (tot > old)  // its phase breakdown (racy between near-equal waves: a diagnostic)
        for (int k = 0; k < kStampCount0; ++k) g_stamp_slowest[k] = acc[k];
    }
  }
};
#else
struct Stamps {
  __device__ void begin() {}
  __device__ void mark(int) {}
  __device__ void count(int, unsigned) {}
  __device__ void note_pairs(unsigned) {}
  __device__ void note_its(unsigned) {}
  __device__ void substep_end(int) {}
  __device__ void note_caps(int, int, int) {}
  __device__ void flush() {}
};
#endif

// ------------------------------------------------------------------------- math
__device__ __forceinline__ void cross3(const float a[3], const float b[3], float o[3]) {
  float x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
__device__ __forceinline__ float dot3(const float a[3], const float b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
__device__ __forceinline__ void qmul(const float a[4], const float b[4], float o[4]) {
  float w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  float x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  float y = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  float z = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  o[0] = w; o[1] = x; o[2] = y; o[3] = z;
}
__device__ __forceinline__ void qmat(const float q[4], float R[9]) {
  float w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1.f - 2.f * (y * y + z * z); R[1] = 2.f * (x * y - w * z); R[2] = 2.f * (x * z + w * y);
  R[3] = 2.f * (x * y + w * z); R[4] = 1.f - 2.f * (x * x + z * z); R[5] = 2.f * (y * z - w * x);
  R[6] = 2.f * (x * z - w * y); R[7] = 2.f * (y * z + w * x); R[8] = 1.f - 2.f * (x * x + y * y);
}
__device__ __forceinline__ void mv3(const float R[9], const float v[3], float o[3]) {
  float x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  float y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  float z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
__device__ __forceinline__ void qnormalize(float q[4]) {
  float r = 1.f / sqrtf(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]);
  q[0] *= r; q[1] *= r; q[2] *= r; q[3] *= r;
}
__device__ __forceinline__ float clampf(float x, float lo, float hi) { return fminf(fmaxf(x, lo), hi); }

// sin/cos with Cody-Waite reduction by pi/2 and Cephes minimax polynomials on [-pi/4, pi/4]
// (<= 2 ulp for the half joint angles and rotation angles seen here, |x| < 1e3; no Payne-Hanek
// slow path, which would otherwise be inlined at each of the ~40 call sites of the kernel).
__device__ __forceinline__ void sincos_r(float x, float* sn, float* cs) {
  const float kf = rintf(x * 0.636619772367581343f);
  const int k = (int)kf;
  float r = fmaf(-kf, 1.57079637050628662f, x);
  r = fmaf(kf, 4.37113900018624283e-8f, r);
  const float z = r * r;
  const float sp = fmaf(fmaf(fmaf(-1.9515295891e-4f, z, 8.3321608736e-3f), z, -1.6666654611e-1f), z * r, r);
  const float cp = fmaf(fmaf(fmaf(fmaf(2.443315711809948e-5f, z, -1.388731625493765e-3f), z, 4.166664568298827e-2f), z,
                             -0.5f), z, 1.f);
  const float s0 = (k & 1) ? cp : sp;
  const float c0 = (k & 1) ? sp : cp;
  *sn = (k & 2) ? -s0 : s0;
  *cs = ((k + 1) & 2) ? -c0 : c0;
}
// tanh: Cephes odd polynomial below 0.625, 1 - 2 / (exp(2|x|) + 1) above (~1e-7 abs)
__device__ __forceinline__ float tanh_r(float x) {
  const float ax = fabsf(x);
  if (ax < 0.625f) {
    const float z = x * x;
    return fmaf(fmaf(fmaf(fmaf(fmaf(-5.70498872745e-3f, z, 2.06390887954e-2f), z, -5.37397155531e-2f), z,
                          1.33314422036e-1f), z, -3.33332819422e-1f), z * x, x);
  }
  const float e = __expf(2.f * fminf(ax, 20.f));
  return copysignf(1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f), x);
}

// device-side counters of one handle
struct Counters {
  uint64_t calls;  // zb_step + zb_reset calls (RNG stream position of resets)
  uint64_t steps;  // zb_step calls (common_step_counter)
  int32_t stage;   // curriculum stage (my_curriculum)
  int32_t changed;  // the last finalize widened the command ranges (manager fixup)
  // v4 command sampling state (resample_commands params, changed by the curricula)
  float vel[2], yaw[2], prob_pos;
  int32_t ring_n, ring_head;  // range_curriculum reward buffers (deque(maxlen=24))
  float ring_vel[ZB_V4_RING], ring_yaw[ZB_V4_RING];
};

__host__ __device__ __forceinline__ uint64_t hash64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// ------------------------------------------------------------------------- state in registers
struct Phys {
  float pos[3], quat[4], lv[3], av[3], jq[ND], jqd[ND];
};

// Non-finite guard: true when any physics state value is inf / NaN (an exponent test on the bits:
// -ffast-math folds isfinite away). The step kernels end such an env's episode as `died` with a
// finite reward and reset it, instead of letting NaN persist in its state (a safety net outside
// the reference's semantics: finite states never take it).
__device__ __forceinline__ bool phys_bad(const Phys& p) {
  unsigned bad = 0u;
  auto chk = [&bad](float x) {
    // through an empty asm: under -ffast-math the compiler may assume x finite and fold the test
    unsigned u = __float_as_uint(x);
    asm volatile("" : "+v"(u));
    bad |= ((u >> 23) & 0xffu) == 0xffu ? 1u : 0u;
  };
#pragma unroll
  for (int a = 0; a < 3; ++a) { chk(p.pos[a]); chk(p.lv[a]); chk(p.av[a]); }
#pragma unroll
  for (int a = 0; a < 4; ++a) chk(p.quat[a]);
#pragma unroll
  for (int j = 0; j < ND; ++j) { chk(p.jq[j]); chk(p.jqd[j]); }
  return bad != 0u;
}
struct Kin {
  float q[NB][4], R[NB][9], p[NB][3];  // p relative to P = root origin
  float ax[ND][3], org[ND][3];
};

__device__ __forceinline__ void fk(MP m, const Phys& s, Kin& k) {
  k.q[0][0] = s.quat[0]; k.q[0][1] = s.quat[1]; k.q[0][2] = s.quat[2]; k.q[0][3] = s.quat[3];
  qnormalize(k.q[0]);
  qmat(k.q[0], k.R[0]);
  k.p[0][0] = k.p[0][1] = k.p[0][2] = 0.f;
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    float qj[4], Rj[9], t[3];
    float jpr[4], jpp[3], jcp[3], jcr[4];
    ldc(jpr, m->joint_parent_rot[j]);
    ldc(jpp, m->joint_parent_pos[j]);
    ldc(jcp, m->joint_child_pos[j]);
    ldc(jcr, m->joint_child_rot[j]);
    qmul(k.q[j], jpr, qj);
    qmat(qj, Rj);
    mv3(k.R[j], jpp, t);
#pragma unroll
    for (int a = 0; a < 3; ++a) { k.org[j][a] = k.p[j][a] + t[a]; k.ax[j][a] = Rj[3 * a + 2]; }
    float sn, cs;
    sincos_r(0.5f * s.jq[j], &sn, &cs);
    const float qz[4] = {cs, 0.f, 0.f, sn};
    float qa[4], Ra[9];
    qmul(qj, qz, qa);
    qmat(qa, Ra);
    mv3(Ra, jcp, t);
#pragma unroll
    for (int a = 0; a < 3; ++a) k.p[j + 1][a] = k.org[j][a] + t[a];
    qmul(qa, jcr, k.q[j + 1]);
    qnormalize(k.q[j + 1]);
    qmat(k.q[j + 1], k.R[j + 1]);
  }
}

// spatial velocities V = [omega; v_P] of all bodies
__device__ __forceinline__ void body_vel(const Kin& k, const Phys& s, float V[NB][6]) {
#pragma unroll
  for (int a = 0; a < 3; ++a) { V[0][a] = s.av[a]; V[0][3 + a] = s.lv[a]; }
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    float oxa[3];
    cross3(k.org[j], k.ax[j], oxa);
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      V[j + 1][a] = V[j][a] + k.ax[j][a] * s.jqd[j];
      V[j + 1][3 + a] = V[j][3 + a] + oxa[a] * s.jqd[j];
    }
  }
}

// ------------------------------------------------------------------------- spatial inertia
struct SI { float m, h[3], I[6]; };  // about P, I = xx yy zz xy xz yz

__device__ __forceinline__ void si_mul(const SI& I, const float V[6], float f[6]) {
  const float* w = V;
  const float* v = V + 3;
  float Iw0 = I.I[0] * w[0] + I.I[3] * w[1] + I.I[4] * w[2];
  float Iw1 = I.I[3] * w[0] + I.I[1] * w[1] + I.I[5] * w[2];
  float Iw2 = I.I[4] * w[0] + I.I[5] * w[1] + I.I[2] * w[2];
  float hv[3], hw[3];
  cross3(I.h, v, hv);
  cross3(I.h, w, hw);
  f[0] = Iw0 + hv[0]; f[1] = Iw1 + hv[1]; f[2] = Iw2 + hv[2];
  f[3] = I.m * v[0] - hw[0]; f[4] = I.m * v[1] - hw[1]; f[5] = I.m * v[2] - hw[2];
}

__device__ __forceinline__ void body_si(MP m, const Kin& k, int b, SI& o) {
  const float* R = k.R[b];
  float c[3];
  float bcom[3], L[6];
  ldc(bcom, m->body_com[b]);
  ldc(L, m->body_inertia[b]);
  mv3(R, bcom, c);
  c[0] += k.p[b][0]; c[1] += k.p[b][1]; c[2] += k.p[b][2];
  const float Il[9] = {L[0], L[3], L[4], L[3], L[1], L[5], L[4], L[5], L[2]};
  float T[9], W[9];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int q = 0; q < 3; ++q) T[3 * r + q] = R[3 * r] * Il[q] + R[3 * r + 1] * Il[3 + q] + R[3 * r + 2] * Il[6 + q];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int q = 0; q < 3; ++q) W[3 * r + q] = T[3 * r] * R[3 * q] + T[3 * r + 1] * R[3 * q + 1] + T[3 * r + 2] * R[3 * q + 2];
  const float mm = m->body_mass[b];
  const float cc = dot3(c, c);
  o.m = mm;
  o.h[0] = mm * c[0]; o.h[1] = mm * c[1]; o.h[2] = mm * c[2];
  o.I[0] = W[0] + mm * (cc - c[0] * c[0]);
  o.I[1] = W[4] + mm * (cc - c[1] * c[1]);
  o.I[2] = W[8] + mm * (cc - c[2] * c[2]);
  o.I[3] = W[1] - mm * c[0] * c[1];
  o.I[4] = W[2] - mm * c[0] * c[2];
  o.I[5] = W[5] - mm * c[1] * c[2];
}

// ------------------------------------------------------------------------- packed lower-triangular 12x12
constexpr int tri(int r, int c) { return r * (r + 1) / 2 + c; }  // r >= c
constexpr int NT = NV * (NV + 1) / 2;

__device__ __forceinline__ void fwd_sub(const float L[NT], const float inv[NV], const float b[NV], float y[NV]) {
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    float t = b[i];
#pragma unroll
    for (int k = 0; k < i; ++k) t -= L[tri(i, k)] * y[k];
    y[i] = t * inv[i];
  }
}
__device__ __forceinline__ void bwd_sub(const float L[NT], const float inv[NV], const float y[NV], float x[NV]) {
#pragma unroll
  for (int i = NV - 1; i >= 0; --i) {
    float t = y[i];
#pragma unroll
    for (int k = i + 1; k < NV; ++k) t -= L[tri(k, i)] * x[k];
    x[i] = t * inv[i];
  }
}
// 12-term dot with a 4-way split accumulation (shorter dependency chain than a serial sum)
__device__ __forceinline__ float dot12(const float a[NV], const float b[NV]) {
  float s0 = a[0] * b[0], s1 = a[1] * b[1], s2 = a[2] * b[2], s3 = a[3] * b[3];
  s0 += a[4] * b[4]; s1 += a[5] * b[5]; s2 += a[6] * b[6]; s3 += a[7] * b[7];
  s0 += a[8] * b[8]; s1 += a[9] * b[9]; s2 += a[10] * b[10]; s3 += a[11] * b[11];
  return (s0 + s1) + (s2 + s3);
}

// Model constants are wave-uniform and re-loaded (scalar loads) where used; routing the pointer
// through an empty asm keeps the compiler from hoisting hundreds of them out of the substep loop
// into long-lived registers.
__device__ __forceinline__ MP opaque(MP m) {
  uint64_t v = (uint64_t)m;
  asm volatile("" : "+s"(v));
  return (MP)v;
}

// ------------------------------------------------------------------------- teams
// Sixteen lanes per env: a team is one 16-lane DPP row (lane = 16 e + s, 4 envs per wave). The
// articulated-body dynamics (FK, RNEA, CRBA, Cholesky) are evaluated redundantly by the team;
// the contact work is split: lane s tests link s against the ground, a sixteenth of the
// self-collision pairs, builds the rows of contact slot s, and in the Gauss-Seidel sweep owns
// whitened coordinate s (s < 12). Row dots are reduced across the team with DPP adds
// (quad_perm, row_half_mirror, row_mirror), which leave all 16 lanes bit-identical sums, so the
// redundant scalar work stays identical across the team.
constexpr int TL = 16;           // lanes per env
#ifndef ZB_WAVES_PER_SIMD
#define ZB_WAVES_PER_SIMD 2
#endif
// The manager kernel needs the explicit bound: left at 1 it takes 256 VGPRs + 4 AGPRs (one wave
// per SIMD); at 2 it fits 256 registers with 16 B/lane of scratch and runs 39 % faster at 8192 envs.
// The other step kernels fit 256 VGPRs without spilling either way (LDS allows two waves).
#ifndef ZB_M_WAVES_PER_SIMD
#define ZB_M_WAVES_PER_SIMD 2
#endif
constexpr int EPW = 4;           // envs per workgroup (one wave)
constexpr int WGT = TL * EPW;    // threads per workgroup
static_assert(WGT <= WAVE, "one wave per workgroup");
// lane c of a team builds / zeroes / maps / forces contact slot c: one slot per lane
static_assert(NCM <= TL, "ZB_MAX_CONTACTS <= 16 (one contact slot per lane of the env's team)");

template <int CTRL>
__device__ __forceinline__ float dppf(float x) {
  // bound_ctrl: an invalid source lane reads 0, the same as keeping old = 0, but the compiler
  // need not materialise old (folds into v_add_f32_dpp / drops the v_mov 0)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
template <int CTRL>
__device__ __forceinline__ int dppi(int x) {
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true);
}
template <int CTRL>
__device__ __forceinline__ int dppz(int x) {  // out-of-row source lanes read 0 (row shifts)
  return __builtin_amdgcn_update_dpp(0, x, CTRL, 0xF, 0xF, true);
}
constexpr int DPP_XOR1 = 0xB1, DPP_XOR2 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140;
constexpr int DPP_BCAST = 0x150, DPP_SHR = 0x110, DPP_SHL = 0x100;  // row_newbcast:k, row_shr:k, row_shl:k

template <int CTRL>
__device__ __forceinline__ float dppzf(float x) {  // out-of-row source lanes read 0 (row shifts)
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, true));
}
// suffix sums over the team: x_b <- sum_{b' >= b} x_b' (lanes past the row contribute 0)
template <int NF>
__device__ __forceinline__ void suffix_sum(float (&x)[NF]) {
#pragma unroll
  for (int a = 0; a < NF; ++a) x[a] += dppzf<DPP_SHL + 1>(x[a]);
#pragma unroll
  for (int a = 0; a < NF; ++a) x[a] += dppzf<DPP_SHL + 2>(x[a]);
#pragma unroll
  for (int a = 0; a < NF; ++a) x[a] += dppzf<DPP_SHL + 4>(x[a]);
}
__device__ __forceinline__ float tsum(float x) {
  // keep x's producer (usually a product) out of the first add: contracted into an fma it would
  // need a separate v_mov_dpp; as a plain add the DPP folds into v_add_f32_dpp
  asm("" : "+v"(x));
  x += dppf<DPP_XOR1>(x);
  x += dppf<DPP_XOR2>(x);
  x += dppf<DPP_HALF_MIRROR>(x);
  return x + dppf<DPP_MIRROR>(x);
}
__device__ __forceinline__ float tmax(float x) {
  x = fmaxf(x, dppf<DPP_XOR1>(x));
  x = fmaxf(x, dppf<DPP_XOR2>(x));
  x = fmaxf(x, dppf<DPP_HALF_MIRROR>(x));
  return fmaxf(x, dppf<DPP_MIRROR>(x));
}
__device__ __forceinline__ int tor(int x) {
  x |= dppi<DPP_XOR1>(x);
  x |= dppi<DPP_XOR2>(x);
  x |= dppi<DPP_HALF_MIRROR>(x);
  return x | dppi<DPP_MIRROR>(x);
}
__device__ __forceinline__ int tscan(int x) {  // inclusive prefix sum over the team
  x += dppz<DPP_SHR + 1>(x);
  x += dppz<DPP_SHR + 2>(x);
  x += dppz<DPP_SHR + 4>(x);
  return x + dppz<DPP_SHR + 8>(x);
}
template <int K>
__device__ __forceinline__ float tb(float x) { return dppf<DPP_BCAST + K>(x); }  // lane K of the team
template <int K>
__device__ __forceinline__ int tbi(int x) { return dppi<DPP_BCAST + K>(x); }

// tanh of the env's raw actions (_pre_physics_step's torch.tanh, v2.py:276-287), correctly rounded: lane
// j < ND evaluates action j in double and the team broadcasts, as the oracle's (real)tanh((double)a).
// The single-precision polynomial (tanh_r, ~1e-7) doubled the device's median error against exact
// arithmetic on p_delta / actions; this costs one double tanh per lane per step.
// tanh in double, rounded to float: expm1(2|x|) by Cody-Waite reduction (n = rint(y / ln 2)) and the
// Taylor series of e^r - 1 to r^13 (|r| <= ln 2 / 2: < 1e-17 relative), then em1 / (em1 + 2) with
// one Newton step on the reciprocal (no cancellation for small |x|: em1 = q there)
__device__ __forceinline__ float tanh_f64(float xf) {
  const double y = 2.0 * fmin(fabs((double)xf), 20.0);
  const double n = rint(y * 1.4426950408889634074);
  const double r = fma(-n, 1.90821492927058770002e-10, fma(-n, 6.93147180369123816490e-01, y));
  double p = 1.0 / 6227020800.0;
  p = fma(p, r, 1.0 / 479001600.0);
  p = fma(p, r, 1.0 / 39916800.0);
  p = fma(p, r, 1.0 / 3628800.0);
  p = fma(p, r, 1.0 / 362880.0);
  p = fma(p, r, 1.0 / 40320.0);
  p = fma(p, r, 1.0 / 5040.0);
  p = fma(p, r, 1.0 / 720.0);
  p = fma(p, r, 1.0 / 120.0);
  p = fma(p, r, 1.0 / 24.0);
  p = fma(p, r, 1.0 / 6.0);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  const double q = p * r;  // e^r - 1
  const double em1 = n == 0.0 ? q : ldexp(1.0 + q, (int)n) - 1.0;
  const double d = em1 + 2.0;
  double rc = __builtin_amdgcn_rcp(d);
  rc = fma(rc, fma(-d, rc, 1.0), rc);
  rc = fma(rc, fma(-d, rc, 1.0), rc);
  return copysignf((float)(em1 * rc), xf);
}
__device__ __forceinline__ void actions_tanh(const float* __restrict__ act, int i, int s, float out[ND]) {
  // (every lane evaluates one -- lanes past ND repeat action 0 -- so no divergent branch splits the
  // prologue)
  const float mine = tanh_f64(act[(size_t)i * ZB_ACT_DIM + (s < ND ? s : 0)]);
  out[0] = tb<0>(mine); out[1] = tb<1>(mine); out[2] = tb<2>(mine);
  out[3] = tb<3>(mine); out[4] = tb<4>(mine); out[5] = tb<5>(mine);
}

// position of the r-th (0-based) set bit of m (r < popcount(m)): binary search on popcounts
__device__ __forceinline__ int nth_set_bit(unsigned long long m, int r) {
  int pos = 0;
#pragma unroll
  for (int w = 32; w >= 1; w >>= 1) {
    const unsigned long long low = m & ((1ull << w) - 1ull);
    const int c = __popcll(low);
    const bool up = r >= c;
    r -= up ? c : 0;
    pos += up ? w : 0;
    m = up ? m >> w : low;
  }
  return pos;
}

// Workgroups of the step / substep kernels are exactly one wave: LDS operations of a wave execute
// in order, so cross-lane LDS hand-offs need only a compiler-level fence (no s_barrier, and no
// wait on outstanding global loads/stores, which __syncthreads would add).
__device__ __forceinline__ void wave_sync() {
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  __builtin_amdgcn_wave_barrier();
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
}

// Workgroup b runs on XCD b % 8 (round-robin dispatch). Give the workgroups of one XCD a
// contiguous range of envs so that the 64-B segments of a state field that neighbouring
// workgroups touch share that XCD's L2 (otherwise each line is fetched once per XCD).
constexpr int NXCD = 8;
__device__ __forceinline__ int xcd_block(int b, int nb) {
  if (nb % NXCD) return b;
  return (b % NXCD) * (nb / NXCD) + b / NXCD;
}

// Device-side per-link collision table (built by zb_create), float4-aligned for per-lane loads:
// [0] bounding sphere, [1+3ci..3+3ci] circle ci: C, E1, E2 (body frame), [7 + ci] core circle ci
// {centre, semi-axis scale (r - kCoreM) / r}, [9] bounding sphere of the two circles (midpoint of
// the centres, max |C - mid| + r + 1 um) for the self-collision broadphase.
// After the NL links: the self-pair list as ints (16 la + lb), then the default-pose constants.
constexpr int LINK4 = 10;
constexpr int NPAIR = (NL - 1) * (NL - 2) / 2;  // non-adjacent link pairs (55), checked by zb_create
constexpr int PAIRS_PER_LANE = (NPAIR + TL - 1) / TL;
// default pose (zb_derive_kernel): feet positions, base quat, base quat relative to the root, feet
// positions in the root frame (at the default joint positions)
constexpr int DFLT_OFF = NL * LINK4 + (NPAIR + 3) / 4;
constexpr int JT_OFF = DFLT_OFF + 6;  // joints: {jpr}, {jpp}, {jcp}, {jcr}, {a_local = R(jpr) z}
constexpr int BT_OFF = JT_OFF + ND * 5;  // bodies: {com, mass}, {Ixx, Iyy, Izz, Ixy}, {Ixz, Iyz, 0, 0}
constexpr int LNK4 = BT_OFF + NB * 3;

// Candidate list in canonical order: ground (link by link, <= 4 each), then self candidates in
// (pair, sphere a, sphere b) order, at most NSELF. More than NCM candidates: the NCM smallest by
// (sep, canonical index) are kept; kept contacts are solved in canonical order (= oracle detect).
constexpr int NCAND = NL * 4 + NSELF;

// LDS layout of one workgroup (EPW envs), float4 units. Phase-disjoint buffers share storage so
// that a workgroup needs <= 20 KB: with 253 VGPRs that lets two waves share a SIMD (8 per CU)
// once a launch has more than one wave per SIMD (N > 4096 envs).
//   region U (per substep: detection -> contact rows -> PGS; then the epilogue)
//     CAND  [EPW][NCAND][2]  candidates {x, sep}, {n, code = 16 la + lb + 1}     detection .. row read
//     MAP   [EPW][NCM] int   overflow only: solver slot -> candidate position     detection .. row read
//     KEEP  [EPW][NCAND] u8  overflow only: kept flags                            detection
//     YG    [NCM][EPW*NV+1]  granule (e, d) of slot c: {Y0[d], Y1[d], Y2[d], 0};  row write .. PGS
//                            the trailing granule of a slot is zero (lanes d >= NV read it)
//     STG   [EPW][STG_LEN] f32, LOGR [EPW][ACC] f32                              epilogue only
//   region V
//     CAP   [NL][2][EPW]     world core capsules {circle centre, core radius}     detection only
//     stash [WGT][2]         M rows of the joint columns (saturated drives)       Cholesky .. re-solve
//     AUX   [NCM][2][EPW]    {invm0, invm1, invm2, vmin invm0}, {c01 invm1, c02 invm2, mu_s, mu_d}
//     LAM   [NCM][EPW]       contact impulses {ln, l1, l2, 0}                     row write .. sensor
//     FRC   [NCM][EPW]       contact normal + code (row builder), then force {f, code} (sensor)
//   BODY  [NB][4][EPW]      body poses {R row 0, p.x}, {R row 1, p.y}, {R row 2, p.z}, {quat}
//   JNT   [ND][3][EPW]      joints {a, o.x}, {o x a, o.y}, {o.z, -}
//   LNK   [LNK4 - NL*LINK4] pair codes, default pose, joint / body tables (the per-link collision
//                           table is read from global memory: L1-resident, 3 KB)
//   PRE   [EPW][PRE4]       prologue results parked across the physics
//   FRIC  [EPW][2][NL] f32  per-link static / dynamic friction coefficients (standup, manager)
//   SENS  [EPW][MAXSUB][2]  per-substep contact-sensor record {fz0, fz1, |F0|, |F1|}, {undesired max |F|}
//   CARRY [EPW][CARRY_W] f32  the env's MDP state rows, prefetched in the prologue (carry_prefetch)
#ifndef ZB_YG_PAD
#define ZB_YG_PAD 1
#endif
constexpr int CAND_OFF = 0;
constexpr int MAP_OFF = CAND_OFF + EPW * NCAND * 2;
constexpr int KEEP_OFF = MAP_OFF + (EPW * NCM + 3) / 4;
constexpr int CAND_END = KEEP_OFF + (EPW * NCAND + 15) / 16;
constexpr int YG_OFF = 0;
// contact-row slot stride: EPW * NV granules + the zero granule. The PGS reads slot c as one
// contiguous run (lane (e, d) -> granule e NV + d); the stride is odd, so the contact-row
// builder's writes (lane c writes granules d = 0..NV-1 of slot c) do not land on one bank group.
constexpr int YGS = EPW * NV + 1;
constexpr int YG_END = YG_OFF + NCM * YGS;
constexpr int U_END = CAND_END > YG_END ? CAND_END : YG_END;
// per-slot records written by lane c (slot c) and read team-uniformly: slot strides padded
constexpr int AUX_S = 2 * EPW + ZB_YG_PAD, LAM_S = EPW + ZB_YG_PAD;
constexpr int V_OFF = U_END;
constexpr int UB_OFF = V_OFF;       // detection only
constexpr int STASH_OFF = V_OFF;    // Cholesky .. saturated re-solve (after detection, before rows)
constexpr int AUX_OFF = V_OFF;
constexpr int LAM_OFF = AUX_OFF + NCM * AUX_S;
constexpr int FRC_OFF = LAM_OFF + NCM * LAM_S;
constexpr int V_END = FRC_OFF + NCM * LAM_S;
static_assert(2 * NL * EPW <= NCM * AUX_S + NCM * LAM_S, "CAP fits below FRC");
static_assert(2 * WGT <= NCM * AUX_S + NCM * LAM_S, "stash fits below FRC");
constexpr int BODY_OFF = V_END;
// per-body / per-joint strides padded by one granule: lane b of a team publishes body b (joint b),
// so unpadded strides of 16 (12) granules would put the team's writes on the same banks
constexpr int BODY_S = 4 * EPW + ZB_YG_PAD, JNT_S = 3 * EPW + ZB_YG_PAD;
constexpr int JNT_OFF = BODY_OFF + NB * BODY_S;
constexpr int LNK_G = NL * LINK4;      // link-table granules read from global memory
constexpr int LNK_OFF = JNT_OFF + ND * JNT_S - LNK_G;  // lds[LNK_OFF + t] = links[t] for t >= LNK_G
constexpr int PRE_OFF = LNK_OFF + LNK4;  // [EPW] Pre records (prologue -> MDP)
constexpr int PRE4 = 8;                   // float4 per Pre record (30 floats)
constexpr int FRIC_OFF = PRE_OFF + EPW * PRE4;  // [EPW][2][NL] f32 per-link static, dynamic friction
constexpr int MAXSUB = 8;                 // decimation limit (zb_create checks)
constexpr int SENS_OFF = FRIC_OFF + (EPW * 2 * NL + 3) / 4;
constexpr int LOGR_W = ZB_MAX_REWARD_TERMS + 8;  // = ACC (episode-log entries, defined with the step kernels)
constexpr int CARRY0 = ZB_S_P_DELTA, CARRY_W = 64;  // state rows [CARRY0, CARRY0 + CARRY_W)
constexpr int CARRY_OFF = SENS_OFF + EPW * MAXSUB * 2;
constexpr int LDS4 = CARRY_OFF + EPW * CARRY_W / 4;
constexpr int STG_LEN = 88 + 25 + 3;  // >= max state dim + max obs dim + {reward, term, trunc}
constexpr int LOGR_OFF = (EPW * STG_LEN + 3) / 4;  // region U, after STG
static_assert(LOGR_OFF + EPW * LOGR_W / 4 <= U_END, "STG + LOGR fit region U");

// prologue results the MDP reads after the physics (parked in LDS across the substeps)
struct Pre {
  float a_now[ND], pdel[ND], r_pre[5];
  float base_y, base_z, heading, fwd[3], feet[2][3], action_rate;
};

static_assert(sizeof(Pre) <= 16 * 8, "Pre fits PRE4 granules");

struct Q {
  float4* b;
  int lane, e, s;
  const float4* gl;   // per-link collision table (global memory)
  // this lane's contact-row granule in a slot (the zero granule for s >= NV)
  __device__ __forceinline__ int ygl() const { return s < NV ? NV * e + s : EPW * NV; }
  __device__ __forceinline__ float4& yg(const float4* y, int c) const { return const_cast<float4*>(y)[c * YGS]; }
  __device__ __forceinline__ float4& yg_at(int c, int d) const { return b[YG_OFF + c * YGS + NV * e + d]; }
  __device__ __forceinline__ float4& yg_zero(int c) const { return b[YG_OFF + c * YGS + EPW * NV]; }
  __device__ __forceinline__ float4& aux(int c, int h) const { return b[AUX_OFF + c * AUX_S + h * EPW + e]; }
  __device__ __forceinline__ float4& lam(int c) const { return b[LAM_OFF + c * LAM_S + e]; }
  __device__ __forceinline__ float4& frc(int c) const { return b[FRC_OFF + c * LAM_S + e]; }
  __device__ __forceinline__ float4& cand(int p, int h) const { return b[CAND_OFF + (e * NCAND + p) * 2 + h]; }
  __device__ __forceinline__ int& map(int c) const { return reinterpret_cast<int*>(b + MAP_OFF)[e * NCM + c]; }
  __device__ __forceinline__ unsigned char& keep(int p) const { return reinterpret_cast<unsigned char*>(b + KEEP_OFF)[e * NCAND + p]; }
  __device__ __forceinline__ float4& body(int bb, int r) const { return b[BODY_OFF + bb * BODY_S + r * EPW + e]; }
  __device__ __forceinline__ float4& frame(int bb, int r) const { return body(bb, r); }
  __device__ __forceinline__ float4& jnt(int j, int r) const { return b[JNT_OFF + j * JNT_S + r * EPW + e]; }
  __device__ __forceinline__ const float4* jtab(int j) const { return b + LNK_OFF + JT_OFF + j * 5; }
  __device__ __forceinline__ const float4* btab(int bb) const { return b + LNK_OFF + BT_OFF + bb * 3; }
  __device__ __forceinline__ float4& cap(int l, int k) const { return b[UB_OFF + (2 * l + k) * EPW + e]; }
  __device__ __forceinline__ const float4* link(int l) const { return gl + l * LINK4; }
  __device__ __forceinline__ int pair_code(int p) const { return reinterpret_cast<const int*>(b + LNK_OFF + NL * LINK4)[p]; }
  __device__ __forceinline__ const float4* dflt() const { return b + LNK_OFF + DFLT_OFF; }
  __device__ __forceinline__ Pre& pre() const { return *reinterpret_cast<Pre*>(b + PRE_OFF + e * PRE4); }
  __device__ __forceinline__ float& fric(int l) const { return reinterpret_cast<float*>(b + FRIC_OFF)[e * 2 * NL + l]; }
  __device__ __forceinline__ float& fricd(int l) const { return reinterpret_cast<float*>(b + FRIC_OFF)[e * 2 * NL + NL + l]; }
  __device__ __forceinline__ float4& sens(int k, int h) const { return b[SENS_OFF + (e * MAXSUB + k) * 2 + h]; }
  __device__ __forceinline__ float& stg(int k) const;  // epilogue staging row of this env (staged_store)
  __device__ __forceinline__ float* logr(int ee) const { return reinterpret_cast<float*>(b + LOGR_OFF) + ee * LOGR_W; }
  __device__ __forceinline__ float* carry() const { return reinterpret_cast<float*>(b + CARRY_OFF) + e * CARRY_W; }
};

__device__ __forceinline__ Q make_q(float4* lds, int lane, const float4* links) {
  const int e = lane / TL, s = lane % TL;
  return Q{lds, lane, e, s, links};
}

__device__ __forceinline__ void read_frame(const Q& q, int body, float R[9], float p[3]) {
  const float4 a = q.frame(body, 0), b = q.frame(body, 1), c = q.frame(body, 2);
  R[0] = a.x; R[1] = a.y; R[2] = a.z; p[0] = a.w;
  R[3] = b.x; R[4] = b.y; R[5] = b.z; p[1] = b.w;
  R[6] = c.x; R[7] = c.y; R[8] = c.z; p[2] = c.w;
}
__device__ __forceinline__ void mv3f(const float R[9], const float4 v, float o[3]) {
  const float a[3] = {v.x, v.y, v.z};
  mv3(R, a, o);
}

// ------------------------------------------------------------------------- contact cache
// Persistent self-contact cache (every task's step kernel): rows 4r .. 4r+3 of env i hold
// {n, code} of the env's r-th kept self contact of the previous step's last substep (code -1:
// none), so the first substep's GJK is warm-started like the later ones. Lane s of the team owns
// row s. Invalidated by set_state, resets and the in-kernel auto-reset.
static_assert(ZB_WARM_ROWS == TL, "one cache row per lane of the team");
__device__ __forceinline__ float wc_invalid(int s) { return (s & 3) == 3 ? -1.f : 0.f; }
// the cache into FRC slots 0 .. ZB_WARM_SLOTS-1 (the GJK warm-start lookup), the other slots empty
__device__ __forceinline__ void wc_load(const Q& q, const float* __restrict__ wc, int N, int i) {
  const float v = wc[(unsigned)(q.s * N + i)];  // (32-bit index: N * ZB_WARM_ROWS < 2^32)
  if (q.s < NCM) q.frc(q.s) = make_float4(0.f, 0.f, 0.f, -1.f);
  wave_sync();
  reinterpret_cast<float*>(&q.frc(q.s >> 2))[q.s & 3] = v;
}
// this lane's cache row after the last substep: FRC holds its kept contacts {n, code} by slot
__device__ __forceinline__ float wc_extract(const Q& q) {
  const float4 f = q.frc(q.s < NCM ? q.s : 0);
  bool self = q.s < NCM && f.w >= 1.f && (((int)f.w) & 15) != 0;  // ground codes: 16 l
  // one entry per pair: a face manifold's points share the pair's normal (= oracle wc_store)
#pragma unroll
  for (int c = 0; c < NCM - 1; ++c) self = self & !((c < q.s) & (q.frc(c).w == f.w));  // (bitwise: no branches)
  const unsigned M = (unsigned)(__ballot(self) >> (TL * q.e)) & 0xffffu;
  const int r = q.s >> 2;
  float v = wc_invalid(q.s);
  if (r < __popc(M)) v = reinterpret_cast<const float*>(&q.frc(nth_set_bit(M, r)))[q.s & 3];
  return v;
}
__global__ void zb_wc_fill_kernel(int N, float* __restrict__ wc, const int32_t* __restrict__ ids, int n) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n * ZB_WARM_ROWS) return;
  const int k = t / ZB_WARM_ROWS, r = t % ZB_WARM_ROWS;
  const int e = ids ? ids[k] : k;
  if (e >= 0 && e < N) wc[(size_t)r * N + e] = wc_invalid(r);
}

// ------------------------------------------------------------------------- team kinematics
// FK as a parallel prefix over the team: lane 0 holds the root (q0, 0), lane b >= 1 the local
// transform of joint b-1, M = (jpr * qz(q) * jcr, jpp + rot(jpr * qz(q), jcp)); three DPP row
// shifts (Hillis-Steele, composition (q1, t1) o (q2, t2) = (q1 q2, t1 + rot(q1, t2))) leave body
// b's pose in lane b. Lane b then publishes body b (frame + quaternion) and joint b's axis /
// origin / motion subspace to LDS and, for the dynamics, keeps body b's spatial inertia about P
// and joint b's motion subspace in registers.
__device__ __forceinline__ void qrot(const float q[4], const float v[3], float o[3]) {
  // v + 2 w (u x v) + 2 u x (u x v), u = q.xyz
  const float u[3] = {q[1], q[2], q[3]};
  float t[3];
  cross3(u, v, t);
  t[0] *= 2.f; t[1] *= 2.f; t[2] *= 2.f;
  float ut[3];
  cross3(u, t, ut);
  o[0] = v[0] + q[0] * t[0] + ut[0];
  o[1] = v[1] + q[0] * t[1] + ut[1];
  o[2] = v[2] + q[0] * t[2] + ut[2];
}
template <int D>
__device__ __forceinline__ void fk_scan_step(float qv[4], float tv[3], int lane_b) {
  float qs[4], ts[3];
#pragma unroll
  for (int a = 0; a < 4; ++a) qs[a] = dppf<DPP_SHR + D>(qv[a]);
#pragma unroll
  for (int a = 0; a < 3; ++a) ts[a] = dppf<DPP_SHR + D>(tv[a]);
  // every lane composes, the lanes below D keep theirs (selects: a divergent branch here cost more
  // in exec-mask instructions than the selects)
  float qn[4], rt[3];
  qmul(qs, qv, qn);
  qrot(qs, tv, rt);
  const bool on = lane_b >= D;
#pragma unroll
  for (int a = 0; a < 4; ++a) qv[a] = on ? qn[a] : qv[a];
#pragma unroll
  for (int a = 0; a < 3; ++a) tv[a] = on ? ts[a] + rt[a] : tv[a];
}

template <bool kInertia>
__device__ __forceinline__ void fk_team(const Phys& s, const Q& q, SI& Ib, float (&Sown)[6]) {
  const int b = q.s;
  if (kInertia) {
    Ib.m = 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) Ib.h[a] = 0.f;
#pragma unroll
    for (int a = 0; a < 6; ++a) { Ib.I[a] = 0.f; Sown[a] = 0.f; }
  }
  float qv[4], tv[3] = {0.f, 0.f, 0.f};
  if (b == 0) {
    qv[0] = s.quat[0]; qv[1] = s.quat[1]; qv[2] = s.quat[2]; qv[3] = s.quat[3];
    qnormalize(qv);
  } else {
    const int j = b <= ND ? b - 1 : ND - 1;
    // select this lane's joint angle with v_cndmask (values pinned in registers first, so the
    // select chain is not folded into a dynamically indexed load from a stack copy of the state)
    float jqv[ND];
#pragma unroll
    for (int k = 0; k < ND; ++k) {
      jqv[k] = s.jq[k];
      asm volatile("" : "+v"(jqv[k]));
    }
    float qj = jqv[0];
#pragma unroll
    for (int k = 1; k < ND; ++k) qj = j == k ? jqv[k] : qj;
    const float4* J = q.jtab(j);
    const float4 jpr = J[0], jpp = J[1], jcp = J[2], jcr = J[3];
    float sn, cs;
    sincos_r(0.5f * qj, &sn, &cs);
    const float pr[4] = {jpr.x, jpr.y, jpr.z, jpr.w}, qz[4] = {cs, 0.f, 0.f, sn}, cr[4] = {jcr.x, jcr.y, jcr.z, jcr.w};
    float qa[4], t[3];
    qmul(pr, qz, qa);
    const float cp[3] = {jcp.x, jcp.y, jcp.z};
    qrot(qa, cp, t);
    tv[0] = jpp.x + t[0]; tv[1] = jpp.y + t[1]; tv[2] = jpp.z + t[2];
    qmul(qa, cr, qv);
  }
  fk_scan_step<1>(qv, tv, b);
  fk_scan_step<2>(qv, tv, b);
  fk_scan_step<4>(qv, tv, b);
  if (b < NB) {
    qnormalize(qv);
    float R[9];
    qmat(qv, R);
    q.body(b, 0) = make_float4(R[0], R[1], R[2], tv[0]);
    q.body(b, 1) = make_float4(R[3], R[4], R[5], tv[1]);
    q.body(b, 2) = make_float4(R[6], R[7], R[8], tv[2]);
    q.body(b, 3) = make_float4(qv[0], qv[1], qv[2], qv[3]);
    if (b < ND) {  // joint b: parent body b
      const float4* J = q.jtab(b);
      const float4 jpp = J[1], al = J[4];
      float o[3], ax[3], oxa[3];
      mv3f(R, jpp, o);
      o[0] += tv[0]; o[1] += tv[1]; o[2] += tv[2];
      mv3f(R, al, ax);
      cross3(o, ax, oxa);
      q.jnt(b, 0) = make_float4(ax[0], ax[1], ax[2], o[0]);
      q.jnt(b, 1) = make_float4(oxa[0], oxa[1], oxa[2], o[1]);
      q.jnt(b, 2) = make_float4(o[2], 0.f, 0.f, 0.f);
      if (kInertia) {
        Sown[0] = ax[0]; Sown[1] = ax[1]; Sown[2] = ax[2];
        Sown[3] = oxa[0]; Sown[4] = oxa[1]; Sown[5] = oxa[2];
      }
    }
    if (kInertia) {  // spatial inertia of body b about P (world axes)
      const float4* B = q.btab(b);
      const float4 cm = B[0], i0 = B[1], i1 = B[2];
      float c[3];
      mv3f(R, cm, c);
      c[0] += tv[0]; c[1] += tv[1]; c[2] += tv[2];
      const float Il[9] = {i0.x, i0.w, i1.x, i0.w, i0.y, i1.y, i1.x, i1.y, i0.z};
      float T[9], W[9];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k) T[3 * r + k] = R[3 * r] * Il[k] + R[3 * r + 1] * Il[3 + k] + R[3 * r + 2] * Il[6 + k];
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k) W[3 * r + k] = T[3 * r] * R[3 * k] + T[3 * r + 1] * R[3 * k + 1] + T[3 * r + 2] * R[3 * k + 2];
      const float mm = cm.w;
      const float cc = dot3(c, c);
      Ib.m = mm;
      Ib.h[0] = mm * c[0]; Ib.h[1] = mm * c[1]; Ib.h[2] = mm * c[2];
      Ib.I[0] = W[0] + mm * (cc - c[0] * c[0]);
      Ib.I[1] = W[4] + mm * (cc - c[1] * c[1]);
      Ib.I[2] = W[8] + mm * (cc - c[2] * c[2]);
      Ib.I[3] = W[1] - mm * c[0] * c[1];
      Ib.I[4] = W[2] - mm * c[0] * c[2];
      Ib.I[5] = W[5] - mm * c[1] * c[2];
    }
  }
}

__device__ __forceinline__ void fk_team_pose(const Phys& s, const Q& q) {
  SI dummy;
  float ds[6];
  fk_team<false>(s, q, dummy, ds);
}

__device__ __forceinline__ void read_S(const Q& q, float S[ND][6]) {
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const float4 g0 = q.jnt(j, 0), g1 = q.jnt(j, 1);
    S[j][0] = g0.x; S[j][1] = g0.y; S[j][2] = g0.z;
    S[j][3] = g1.x; S[j][4] = g1.y; S[j][5] = g1.z;
  }
}

// joint motion subspaces S_j = [a_j; o_j x a_j] and origins o_j (relative to P) from LDS
__device__ __forceinline__ void read_joints(const Q& q, float S[ND][6], float org[ND][3]) {
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const float4 g0 = q.jnt(j, 0), g1 = q.jnt(j, 1), g2 = q.jnt(j, 2);
    S[j][0] = g0.x; S[j][1] = g0.y; S[j][2] = g0.z;
    S[j][3] = g1.x; S[j][4] = g1.y; S[j][5] = g1.z;
    org[j][0] = g0.w; org[j][1] = g1.w; org[j][2] = g2.x;
  }
}

__device__ __forceinline__ bool opaque_true() {  // true, unknown to the optimiser
  int one = 1;
  asm volatile("" : "+s"(one));
  return one != 0;
}

template <class T>
__device__ __forceinline__ T* opaque_ptr(T* p) {
  asm volatile("" : "+v"(p));
  return p;
}

// ------------------------------------------------------------------------- contacts
// Self collision: GJK distance between the core hulls of a link pair (world frame, relative to P).
struct Hull {
  float c[2][3], e1[2][3], e2[2][3];  // core circles: centre, semi-axes (radius baked in)
};
__device__ __forceinline__ void world_hull(const Q& q, int l, Hull& h) {
  float R[9], p[3];
  read_frame(q, link_body(l), R, p);
  const float4* L = q.link(l);
#pragma unroll
  for (int ci = 0; ci < 2; ++ci) {
    const float4 cc = L[7 + ci];
    float4 e1 = L[2 + 3 * ci], e2 = L[3 + 3 * ci];
    e1.x *= cc.w; e1.y *= cc.w; e1.z *= cc.w;
    e2.x *= cc.w; e2.y *= cc.w; e2.z *= cc.w;
    mv3f(R, cc, h.c[ci]);
    h.c[ci][0] += p[0]; h.c[ci][1] += p[1]; h.c[ci][2] += p[2];
    mv3f(R, e1, h.e1[ci]);
    mv3f(R, e2, h.e2[ci]);
  }
}
// support point of the hull of the two circles along d (a circle's rim point along d's in-plane
// part; its centre when d is normal to the disk)
// h = the Hull held by the lane at byte address addr (= 4 x lane index), via ds_bpermute; every
// lane of the wave must execute it
__device__ __forceinline__ float bperm(int addr, float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_ds_bpermute(addr, __builtin_bit_cast(int, v)));
}
__device__ __forceinline__ void gather_hull(const Hull& own, int addr, Hull& h) {
#pragma unroll
  for (int ci = 0; ci < 2; ++ci)
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      h.c[ci][k] = bperm(addr, own.c[ci][k]);
      h.e1[ci][k] = bperm(addr, own.e1[ci][k]);
      h.e2[ci][k] = bperm(addr, own.e2[ci][k]);
    }
}
struct SelfContact { float x[3], sep, n[3]; };
// Cheap separation test before GJK: separating-axis gaps along the centre difference and the four
// circle normals (each circle's extent along u is c.u +- |(u.E1, u.E2)|, exact). True when one
// gap exceeds lim = margin + 2 kCoreM: the cores are farther apart than any contact. A rigorous
// bound, so it never drops a contact that GJK would find; on random-action rollouts it decides
// ~99 % of the broadphase pairs without iterating.
// squared distance between the segments p0p1 and q0q1 (xyz of the float4s; closest points by the
// clamped parameters of the two lines, segments of nonzero length)
__device__ __forceinline__ float seg_seg_d2(const float4 p0, const float4 p1, const float4 q0, const float4 q1) {
  const float d1[3] = {p1.x - p0.x, p1.y - p0.y, p1.z - p0.z};
  const float d2[3] = {q1.x - q0.x, q1.y - q0.y, q1.z - q0.z};
  const float r[3] = {p0.x - q0.x, p0.y - q0.y, p0.z - q0.z};
  const float a = fmaxf(dot3(d1, d1), 1e-12f), e = fmaxf(dot3(d2, d2), 1e-12f);
  const float b = dot3(d1, d2), c = dot3(d1, r), f = dot3(d2, r);
  const float den = a * e - b * b;
  float sc = den > 1e-12f * a * e ? clampf((b * f - c * e) / den, 0.f, 1.f) : 0.f;
  float tc = (b * sc + f) / e;
  const float s0 = clampf(-c / a, 0.f, 1.f), s1 = clampf((b - c) / a, 0.f, 1.f);
  sc = tc < 0.f ? s0 : (tc > 1.f ? s1 : sc);
  tc = clampf(tc, 0.f, 1.f);
  float dd[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) dd[k] = r[k] + d1[k] * sc - d2[k] * tc;
  return dot3(dd, dd);
}
__device__ __forceinline__ void hull_extent(const Hull& h, const float u[3], float& lo, float& hi) {
#pragma unroll
  for (int ci = 0; ci < 2; ++ci) {
    const float a = dot3(u, h.e1[ci]), b = dot3(u, h.e2[ci]);
    const float r = sqrtf(fmaf(a, a, b * b)), m = dot3(u, h.c[ci]);
    lo = ci == 0 ? m - r : fminf(lo, m - r);
    hi = ci == 0 ? m + r : fmaxf(hi, m + r);
  }
}
__device__ __forceinline__ bool hulls_separated(const Hull& A, const Hull& B, float lim) {
  float best = -1e30f;
#pragma unroll
  for (int ax = 0; ax < 5; ++ax) {
    float u[3];
    if (ax == 0) {
#pragma unroll
      for (int k = 0; k < 3; ++k) u[k] = 0.5f * (A.c[0][k] + A.c[1][k]) - 0.5f * (B.c[0][k] + B.c[1][k]);
    } else {
      const Hull& H = ax <= 2 ? A : B;
      cross3(H.e1[(ax - 1) & 1], H.e2[(ax - 1) & 1], u);
    }
    const float iu = __builtin_amdgcn_rsqf(fmaxf(dot3(u, u), 1e-30f));
    u[0] *= iu; u[1] *= iu; u[2] *= iu;
    float alo, ahi, blo, bhi;
    hull_extent(A, u, alo, ahi);
    hull_extent(B, u, blo, bhi);
    // gap along u with A on the + side (u), or along -u
    best = fmaxf(best, fmaxf(alo - bhi, blo - ahi));
  }
  return best > lim;
}
// GJK (distance) on the core hulls A, B of a link pair, run by the 4 lanes of a DPP quad: lane j
// holds circle (j & 1) of hull (j >> 1 ? B : A); the simplex is replicated bit-identically in the
// 4 lanes. Simplex = up to three points S0..S2 (with their A-side support points; S0 = the
// newest of the previous iteration); each iteration adds the support point a and takes the
// shortest of the valid affine projections of the subsets containing a, first in the order {a},
// {a,S0}, {a,S1}, {a,S0,S1}, {a,S2}, {a,S0,S2}, {a,S1,S2} (segments, triangles with positive
// barycentrics; the tetrahedron only as the inside test); the new simplex is a, then the used
// points in index order. Per iteration lane j evaluates its circle's support point (the pair of lanes
// of one hull keeps the larger, circle 0 on ties) and two of the candidates (j = 0: {a}, {a,S0};
// 1: {a,S1}, {a,S0,S1}; 2: {a,S2}, {a,S0,S2}; 3: {a,S1,S2}); two DPP butterfly steps pick the
// first shortest in that order. ~2x fewer instructions per iteration than one lane per pair, and
// the 4 quads of a team run up to 4 pairs at once (the usual count of undecided pairs).
// Starts from v0 (B -> A): the pair's contact normal of the previous substep of this step (warm
// start, the first three supports along tilted directions: gjk_tilted) or the hull centre
// difference. Stops when (|v|^2 - v.w) / |v| <= kGjkTol (the distance
// bounds |v| and v.w / |v| agree), after kGjkMaxIt iterations, or as soon as the lower bound
// v.w / |v| exceeds early_margin + 2 kCoreM (no contact; early_margin = margin in the counting
// pass, huge when a counted contact is re-computed). Contact: n = (pa - pb) / d (B -> A),
// sep = d - 2 kCoreM, x = (pa + pb) / 2; overlapping cores: quad_deep. Same statement as the
// oracle's hull_pair.
constexpr int DPP_QB0 = 0x00, DPP_QB2 = 0xAA;  // quad_perm broadcast of quad lane 0 / 2
struct QCircle { float c[3], e1[3], e2[3]; };  // world core circle: centre, semi-axes (radius baked in)
__device__ __forceinline__ void quad_circle(const Q& q, int l, int ci, QCircle& h) {
  float R[9], p[3];
  read_frame(q, link_body(l), R, p);
  const float4* L = q.link(l);
  const float4 cc = L[7 + ci];
  float4 e1 = L[2 + 3 * ci], e2 = L[3 + 3 * ci];
  e1.x *= cc.w; e1.y *= cc.w; e1.z *= cc.w;
  e2.x *= cc.w; e2.y *= cc.w; e2.z *= cc.w;
  mv3f(R, cc, h.c);
  h.c[0] += p[0]; h.c[1] += p[1]; h.c[2] += p[2];
  mv3f(R, e1, h.e1);
  mv3f(R, e2, h.e2);
}
// hull centres (mean of the two circle centres) of A and B in every lane of the quad
__device__ __forceinline__ void quad_centres(const QCircle& h, float ca[3], float cb[3]) {
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float m = 0.5f * (h.c[k] + dppf<DPP_XOR1>(h.c[k]));
    ca[k] = dppf<DPP_QB0>(m);
    cb[k] = dppf<DPP_QB2>(m);
  }
}
// support points pa of A along -v and pb of B along v, in every lane of the quad
__device__ __forceinline__ void quad_support(const QCircle& h, const float v[3], int j, float pa[3], float pb[3]) {
  const float sg = (j & 2) ? 1.f : -1.f;
  const float d[3] = {sg * v[0], sg * v[1], sg * v[2]};
  const float a = dot3(d, h.e1), b = dot3(d, h.e2);
  const float ri = __builtin_amdgcn_rsqf(fmaxf(fmaf(a, a, b * b), 1e-30f));
  float pt[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) pt[k] = h.c[k] + (a * h.e1[k] + b * h.e2[k]) * ri;
  const float val = dot3(d, pt), pv = dppf<DPP_XOR1>(val);
  const bool mine = (j & 1) ? (val > pv) : !(pv > val);  // circle 0 unless circle 1 is strictly larger
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    // (the DPP read as a statement of its own: inside `?:` it would be evaluated only for the
    // lanes with !mine, and bound_ctrl then reads 0 from the masked-off source lanes)
    const float o = dppf<DPP_XOR1>(pt[k]);
    const float sp = mine ? pt[k] : o;
    pa[k] = dppf<DPP_QB0>(sp);
    pb[k] = dppf<DPP_QB2>(sp);
  }
}
// one butterfly step of the candidate selection: take the partner's candidate if it is shorter, or
// as short and earlier in the canonical order (partner_first: the partner's lane is the lower one)
template <int CTRL>
__device__ __forceinline__ void quad_pick(bool partner_first, float& best, float bv[3], float& l1, float& l2,
                                          unsigned& bm) {
  const float ob = dppf<CTRL>(best);
  const bool take = partner_first ? !(ob > best) : (ob < best);
  best = take ? ob : best;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float o = dppf<CTRL>(bv[k]);
    bv[k] = take ? o : bv[k];
  }
  const float o1 = dppf<CTRL>(l1), o2 = dppf<CTRL>(l2);
  const unsigned om = (unsigned)dppi<CTRL>((int)bm);
  l1 = take ? o1 : l1;
  l2 = take ? o2 : l2;
  bm = take ? om : bm;
}
// Overlapping cores (GJK found the origin inside, or a distance below 1 um): the separating-axis
// estimate of the penetration over the hull centre difference and the four circle normals (A c0,
// A c1, B c0, B c1) -- the axis of the largest (least negative) gap, oriented B -> A, is the
// normal and the gap the core separation (clamped to <= 0; >= -the true depth); the point is the
// mean of the hull centres (the deepest points along a circle normal are a whole rim: rounding
// would pick one). Same statement as the oracle's hull_pair.
__device__ __forceinline__ void quad_deep(const QCircle& h, int j, float n[3], float& sep, float x[3]) {
  float ca[3], cb[3], cn[3];
  quad_centres(h, ca, cb);
  cross3(h.e1, h.e2, cn);  // this lane's circle normal
  float best = -1e30f, nb[3] = {0.f, 0.f, 1.f};
#pragma unroll
  for (int ax = 0; ax < 5; ++ax) {
    float u[3];
#pragma unroll
    for (int k = 0; k < 3; ++k)
      u[k] = ax == 0 ? ca[k] - cb[k]
                     : (ax == 1 ? dppf<DPP_QB0>(cn[k]) : (ax == 2 ? dppf<0x55>(cn[k]) : (ax == 3 ? dppf<DPP_QB2>(cn[k]) : dppf<0xFF>(cn[k]))));
    const float uu = dot3(u, u);
    const float iu = __builtin_amdgcn_rsqf(fmaxf(uu, 1e-30f));
    u[0] *= iu; u[1] *= iu; u[2] *= iu;
    const float a = dot3(u, h.e1), b = dot3(u, h.e2);
    const float r = sqrtf(fmaf(a, a, b * b)), m = dot3(u, h.c);
    const float lo = fminf(m - r, dppf<DPP_XOR1>(m - r)), hi = fmaxf(m + r, dppf<DPP_XOR1>(m + r));
    const float alo = dppf<DPP_QB0>(lo), ahi = dppf<DPP_QB0>(hi), blo = dppf<DPP_QB2>(lo), bhi = dppf<DPP_QB2>(hi);
    const float gp = alo - bhi, gm = blo - ahi, g = gp >= gm ? gp : gm;
    const bool take = uu > 1e-24f && g > best;
    best = take ? g : best;
#pragma unroll
    for (int k = 0; k < 3; ++k) nb[k] = take ? (gp >= gm ? u[k] : -u[k]) : nb[k];
  }
  sep = fminf(best, 0.f) - 2.f * kCoreM;
#pragma unroll
  for (int k = 0; k < 3; ++k) { n[k] = nb[k]; x[k] = 0.5f * (ca[k] + cb[k]); }
}
// Warm start (tilt): the first three support directions are v0 tilted by kGjkTilt toward three
// directions 120 degrees apart, so the simplex spans a flat face at once (a support along a face
// normal is an arbitrary rim point); a stop test only along v itself.
__device__ __forceinline__ void gjk_tilted(const float v0[3], int k, float d[3]) {
  const float iv = __builtin_amdgcn_rsqf(dot3(v0, v0));
  const float u[3] = {v0[0] * iv, v0[1] * iv, v0[2] * iv};
  const bool x = fabsf(u[0]) < 0.57f, y = !x && fabsf(u[1]) < 0.57f, z = !x && !y;
  const float ax[3] = {x ? 1.f : 0.f, y ? 1.f : 0.f, z ? 1.f : 0.f};
  float t1[3], t2[3];
  cross3(u, ax, t1);
  const float it1 = __builtin_amdgcn_rsqf(dot3(t1, t1));
  t1[0] *= it1; t1[1] *= it1; t1[2] *= it1;
  cross3(u, t1, t2);
  const float tc = k == 0 ? 1.f : -0.5f, ts = k == 0 ? 0.f : (k == 1 ? 0.8660254f : -0.8660254f);
#pragma unroll
  for (int a = 0; a < 3; ++a) d[a] = u[a] + kGjkTilt * (tc * t1[a] + ts * t2[a]);
}
__device__ __forceinline__ bool gjk_quad(const QCircle& h, int j, const float v0[3], bool tilt, float margin,
                                         float early_margin, SelfContact& out, int& iters) {
  float v[3] = {v0[0], v0[1], v0[2]};
  const float lim = early_margin + 2.f * kCoreM;
  // simplex S0..S2 (n points; S0 = the newest of the previous iteration) with their A-side
  // support points SP and the weights lam of v = sum lam_i S_i
  float S[3][3] = {}, SP[3][3] = {}, lam[3] = {1.f, 0.f, 0.f};
  int n = 0;
  bool overlap = false;
  for (int it = 0; it <= kGjkMaxIt; ++it) {
    iters = it;
    const float vv = dot3(v, v);
    if (n > 0 && vv < 1e-12f) { overlap = true; break; }
    float dir[3] = {v[0], v[1], v[2]};
    const bool tilted = tilt && it < 3;  // (it is wave-uniform)
    if (it < 3 && tilt) gjk_tilted(v0, it, dir);
    float pa[3], aw[3];
    {
      float pb[3];
      quad_support(h, dir, j, pa, pb);
#pragma unroll
      for (int k = 0; k < 3; ++k) aw[k] = pa[k] - pb[k];
    }
    if (n == 0) {  // first point
#pragma unroll
      for (int k = 0; k < 3; ++k) { S[0][k] = aw[k]; SP[0][k] = pa[k]; v[k] = aw[k]; }
      n = 1;
      continue;
    }
    // any direction bounds the distance from below by its support gap dir.w / |dir|: no contact
    // once that exceeds the margin; converged when the gap along v itself is within kGjkTol of |v|
    const float lo = dot3(dir, aw) * __builtin_amdgcn_rsqf(dot3(dir, dir));
    if (lo > lim) return false;
    if (!tilted && sqrtf(vv) - lo <= kGjkTol) break;  // distance bounds within kGjkTol
    // this lane's candidates with the new point a = aw: the segment {a, S_j} (j < 3) and the
    // triangle {a, S_I, S_J} (j = 1: I, J = 0, 1; j = 2: 0, 2; j = 3: 1, 2); lane 0 starts from {a}
    float best = j == 0 ? dot3(aw, aw) : 3.0e38f, bv[3] = {aw[0], aw[1], aw[2]}, l1 = 0.f, l2 = 0.f;
    unsigned bm = 0u;  // simplex points used (bit i: S_i)
    // edge vectors from a: e2 = S_y - a with y = j (lane 3: y = 2) is both the segment's edge and the
    // triangle's second edge (lanes 1, 2 share every term of the segment with their triangle), e1 =
    // S_x - a with x = 0 (lane 3: x = 1)
    float e1[3], e2[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      e1[k] = (j == 3 ? S[1][k] : S[0][k]) - aw[k];
      e2[k] = (j == 0 ? S[0][k] : (j == 1 ? S[1][k] : S[2][k])) - aw[k];
    }
    const float g11 = dot3(e2, e2), r1 = -dot3(aw, e2);
    {
      const float t = r1 / fmaxf(g11, 1e-30f);
      float p[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) p[k] = aw[k] + t * e2[k];
      const float d2 = dot3(p, p);
      const bool ok = (j < n) & (g11 > 1e-20f) & (t > 0.f) & (t < 1.f) & (d2 < best);  // (bitwise: no branches)
      best = ok ? d2 : best;
      bm = ok ? (1u << j) : bm;
      l1 = ok ? t : l1;
#pragma unroll
      for (int k = 0; k < 3; ++k) bv[k] = ok ? p[k] : bv[k];
    }
    {
      const float g00 = dot3(e1, e1), g01 = dot3(e1, e2);
      const float r0 = -dot3(aw, e1);
      const float det = g00 * g11 - g01 * g01;
      const float id = 1.f / (fabsf(det) > 1e-30f ? det : 1e-30f);
      const float ts = (r0 * g11 - r1 * g01) * id, tt = (g00 * r1 - g01 * r0) * id;
      float p[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) p[k] = aw[k] + ts * e1[k] + tt * e2[k];
      const float d2 = dot3(p, p);
      const bool valid = j == 1 ? n >= 2 : ((j >= 2) & (n >= 3));
      const bool ok = valid & (det > 1e-24f * g00 * g11) & (ts > 0.f) & (tt > 0.f) & (ts + tt < 1.f) & (d2 < best);
      best = ok ? d2 : best;
      bm = ok ? (j == 1 ? 3u : (j == 2 ? 5u : 6u)) : bm;
      l1 = ok ? ts : l1;
      l2 = ok ? tt : l2;
#pragma unroll
      for (int k = 0; k < 3; ++k) bv[k] = ok ? p[k] : bv[k];
    }
    quad_pick<DPP_XOR1>((j & 1) != 0, best, bv, l1, l2, bm);
    quad_pick<DPP_XOR2>((j & 2) != 0, best, bv, l1, l2, bm);
    // origin inside the tetrahedron (a, S0, S1, S2)? Only possible when the support gap along dir is
    // not positive: a is the minimiser of dir.x over the Minkowski difference, so lo > 0 puts the
    // origin outside it (the test's 1e-5 barycentric margins cannot pass there either); the gate skips
    // the ~60-instruction test in all but overlapping pairs' iterations (quad-uniform: lo is)
    if (n == 3 && lo <= 0.f) {
      float e0[3], e1[3], e2[3], x12[3];
#pragma unroll
      for (int k = 0; k < 3; ++k) { e0[k] = S[0][k] - aw[k]; e1[k] = S[1][k] - aw[k]; e2[k] = S[2][k] - aw[k]; }
      cross3(e1, e2, x12);
      const float det = dot3(e0, x12);
      // a flat tetrahedron (relative volume below 1e-6) or an origin within 1e-5 of a face is no
      // evidence of an overlap
      if (fabsf(det) > 1e-6f * sqrtf(dot3(e0, e0) * dot3(e1, e1) * dot3(e2, e2))) {
        const float id = 1.f / det;
        float m0[3], x20[3], x01[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) m0[k] = -aw[k];
        cross3(e2, e0, x20);
        cross3(e0, e1, x01);
        const float b0 = dot3(m0, x12) * id, b1 = dot3(m0, x20) * id, b2 = dot3(m0, x01) * id;
        if ((b0 > 1e-5f) & (b1 > 1e-5f) & (b2 > 1e-5f) & (b0 + b1 + b2 < 1.f - 1e-5f)) { overlap = true; break; }
      }
    }
    // new simplex: a first, then the used points in index order
    const int nu = __popc(bm);
    const bool u0 = bm & 1u, u1 = (bm >> 1) & 1u;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const float t1 = u0 ? S[0][k] : (u1 ? S[1][k] : S[2][k]), t1p = u0 ? SP[0][k] : (u1 ? SP[1][k] : SP[2][k]);
      const float t2 = (u0 && u1) ? S[1][k] : S[2][k], t2p = (u0 && u1) ? SP[1][k] : SP[2][k];
      S[2][k] = t2; SP[2][k] = t2p;
      S[1][k] = t1; SP[1][k] = t1p;
      S[0][k] = aw[k]; SP[0][k] = pa[k];
      v[k] = bv[k];
    }
    lam[1] = nu >= 1 ? l1 : 0.f;
    lam[2] = nu >= 2 ? l2 : 0.f;
    lam[0] = 1.f - lam[1] - lam[2];
    n = nu + 1;
  }
  // one exit (a struct written on two paths ends up in scratch memory)
  const float d = sqrtf(dot3(v, v));
  const bool deep = overlap || d < 1e-6f;
  const float id = 1.f / fmaxf(d, 1e-30f);
  float on[3], ox[3], osep = d - 2.f * kCoreM;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    // closest point on A's core: the same weights over the A-side support points
    const float pa = lam[0] * SP[0][k] + (n >= 2 ? lam[1] * SP[1][k] : 0.f) + (n >= 3 ? lam[2] * SP[2][k] : 0.f);
    on[k] = v[k] * id;
    ox[k] = pa - 0.5f * v[k];
  }
  if (deep) quad_deep(h, j, on, osep, ox);  // (quad-uniform)
#pragma unroll
  for (int k = 0; k < 3; ++k) { out.n[k] = on[k]; out.x[k] = ox[k]; }
  out.sep = osep;
  return out.sep < margin;
}

// Self-contact manifold on the pair's quad (cfg.self_manifold; the oracle's face_manifold, PhysX
// PCM keeps up to 4 points per convex pair): each lane tests its core circle as the face of its
// hull along the pair normal (A: -n, B: +n; the hull's supporting circle with its plane normal
// within 15 degrees); with a face on both sides, lane j evaluates sample j of B's rim carried along
// +n onto A's face plane (side 0) and sample j of A's rim carried along -n onto B's (side 1) -- the
// samples: all four quarter points when the source disk lies inside the target, else the tip toward
// the target centre and the two lens crossings moved 0.03 rad toward it -- kept when the foot lies
// inside the target core disk and the core gap - 2 kCoreM is within the margin. The first 4 kept in
// (side, sample) order form the manifold. Returns its size (0: no face manifold: the GJK contact
// alone); with `write`, sink(rank, {x, sep}) takes each of this lane's kept samples. Quad-uniform
// control flow (DPP within the quad).
constexpr float kFaceCos = 0.9659258262890683f;  // cos 15 deg (= oracle FACE_COS)
constexpr float kFaceInsetC = 0.9995500337489875f, kFaceInsetS = 0.029995500202495664f;  // cos / sin 0.03
constexpr float kRimCos = 0.9961946980917455f, kRimSin = 0.08715574274765817f;  // cos / sin 5 deg (= oracle RIM_COS)

// Rim (ruling) manifold on the pair's quad (cfg.self_manifold 2, no face pair; the oracle's
// rim_manifold): lane j's circle support point along its hull's direction (A: -n, B: +n), the four
// broadcast in the quad; when A's ruling (A c0 -> A c1 supports) and B's lie within 5 degrees of the
// contact plane and of each other: the GJK point with its GJK normal (lane 0 writes it; the pair's
// warm start in the next substep) and the two ends of the rulings' overlap along A's ruling (lanes 1
// and 2), more than 1 mm from the GJK point and within the margin, with the normal made
// perpendicular to A's ruling. Returns the point count (0: no rim pair).
template <class Sink>
__device__ __forceinline__ int quad_rim(const QCircle& h, int j, const SelfContact& sc, float margin, bool write,
                                        Sink sink) {
  const float sgd = (j & 2) ? 1.f : -1.f;
  const float dd[3] = {sgd * sc.n[0], sgd * sc.n[1], sgd * sc.n[2]};
  const float a = dot3(dd, h.e1), b = dot3(dd, h.e2);
  const float ri = __builtin_amdgcn_rsqf(fmaxf(fmaf(a, a, b * b), 1e-30f));
  float p[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) p[k] = h.c[k] + (a * h.e1[k] + b * h.e2[k]) * ri;
  float a0[3], sa[3], b0[3], sb[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float p0 = dppf<0x00>(p[k]), p1 = dppf<0x55>(p[k]), p2 = dppf<0xAA>(p[k]), p3 = dppf<0xFF>(p[k]);
    a0[k] = p0; sa[k] = p1 - p0; b0[k] = p2; sb[k] = p3 - p2;
  }
  const float la = sqrtf(dot3(sa, sa)), lb = sqrtf(dot3(sb, sb));
  if (la < 1e-3f || lb < 1e-3f) return 0;
  if (fabsf(dot3(sa, sc.n)) > kRimSin * la || fabsf(dot3(sb, sc.n)) > kRimSin * lb) return 0;
  if (fabsf(dot3(sa, sb)) < kRimCos * la * lb) return 0;
  const float ila = 1.f / la;
  const float ah[3] = {sa[0] * ila, sa[1] * ila, sa[2] * ila};
  const float na = dot3(sc.n, ah);
  float nr[3] = {sc.n[0] - na * ah[0], sc.n[1] - na * ah[1], sc.n[2] - na * ah[2]};
  const float inr = __builtin_amdgcn_rsqf(fmaxf(dot3(nr, nr), 1e-30f));
  nr[0] *= inr; nr[1] *= inr; nr[2] *= inr;
  const float w0[3] = {b0[0] - a0[0], b0[1] - a0[1], b0[2] - a0[2]};
  const float wg[3] = {sc.x[0] - a0[0], sc.x[1] - a0[1], sc.x[2] - a0[2]};
  const float tb0 = dot3(w0, ah), tb1 = tb0 + dot3(sb, ah), tg = dot3(wg, ah);
  const float lo = fmaxf(0.f, fminf(tb0, tb1)), hi = fminf(la, fmaxf(tb0, tb1));
  const bool span = hi - lo > 1e-3f;
  const float dtb = tb1 - tb0;
  bool ok[2];
  float4 px[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const float t = e ? hi : lo;
    const float ua = t * ila, ub = (t - tb0) / (fabsf(dtb) > 1e-12f ? dtb : 1e-12f);
    float xa[3], xb[3], g[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      xa[k] = a0[k] + ua * sa[k];
      xb[k] = b0[k] + ub * sb[k];
      g[k] = xa[k] - xb[k];
    }
    const float sep = dot3(g, nr) - 2.f * kCoreM;
    ok[e] = span && fabsf(t - tg) > 1e-3f && sep < margin;
    px[e] = make_float4(0.5f * (xa[0] + xb[0]), 0.5f * (xa[1] + xb[1]), 0.5f * (xa[2] + xb[2]), sep);
  }
  if (write) {
    if (j == 0) sink(0, make_float4(sc.x[0], sc.x[1], sc.x[2], sc.sep), sc.n);  // (GJK's normal: the warm start)
    if (j == 1 && ok[0]) sink(1, px[0], nr);
    if (j == 2 && ok[1]) sink(ok[0] ? 2 : 1, px[1], nr);
  }
  return 1 + (ok[0] ? 1 : 0) + (ok[1] ? 1 : 0);
}

// Ruling on a face (cfg.self_manifold 3; the oracle's rim_face_manifold): exactly one hull presents a
// face (fm: the face mask of quad_manifold; uo / r: this lane's circle normal oriented along its
// hull's direction and its core radius), the other its ruling within 5 degrees of the contact plane
// (the segment between its two circles' support points): the GJK point (lane 0, GJK's normal) and
// the two ends of the ruling's stretch over the face's core disk (lanes 1 and 2), more than 1 mm
// from the GJK point along the ruling and within the margin, with the face's normal (B -> A) and the
// end's height above the face plane minus 2 kCoreM. Returns the point count (0: not this case).
template <class Sink>
__device__ __forceinline__ int quad_rimface(const QCircle& h, int j, const SelfContact& sc, float margin, bool write,
                                            Sink sink, int fm, const float uo[3], float r) {
  const float sgd = (j & 2) ? 1.f : -1.f;
  const float dd[3] = {sgd * sc.n[0], sgd * sc.n[1], sgd * sc.n[2]};
  const float a = dot3(dd, h.e1), b = dot3(dd, h.e2);
  const float ri = __builtin_amdgcn_rsqf(fmaxf(fmaf(a, a, b * b), 1e-30f));
  float p[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) p[k] = h.c[k] + (a * h.e1[k] + b * h.e2[k]) * ri;
  const bool fa = (fm & 3) != 0;
  const bool l1 = fa ? (fm & 1) == 0 : (fm & 4) == 0;  // the face on the second circle of its hull
  float cf[3], uf[3], r0[3], sv[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float c0 = dppf<0x00>(h.c[k]), c1 = dppf<0x55>(h.c[k]), c2 = dppf<0xAA>(h.c[k]), c3 = dppf<0xFF>(h.c[k]);
    const float u0 = dppf<0x00>(uo[k]), u1 = dppf<0x55>(uo[k]), u2 = dppf<0xAA>(uo[k]), u3 = dppf<0xFF>(uo[k]);
    const float p0 = dppf<0x00>(p[k]), p1 = dppf<0x55>(p[k]), p2 = dppf<0xAA>(p[k]), p3 = dppf<0xFF>(p[k]);
    cf[k] = fa ? (l1 ? c1 : c0) : (l1 ? c3 : c2);
    uf[k] = fa ? (l1 ? u1 : u0) : (l1 ? u3 : u2);
    r0[k] = fa ? p2 : p0;                 // the other hull's ruling
    sv[k] = fa ? p3 - p2 : p1 - p0;
  }
  const float rr0 = dppf<0x00>(r), rr1 = dppf<0x55>(r), rr2 = dppf<0xAA>(r), rr3 = dppf<0xFF>(r);
  const float rf = fa ? (l1 ? rr1 : rr0) : (l1 ? rr3 : rr2);
  const float ls = sqrtf(dot3(sv, sv));
  if (ls < 1e-3f || fabsf(dot3(sv, sc.n)) > kRimSin * ls) return 0;
  const float sg = fa ? -1.f : 1.f;
  const float nr[3] = {sg * uf[0], sg * uf[1], sg * uf[2]};  // B -> A
  float q0[3], qs[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) q0[k] = r0[k] - cf[k];
  const float q0u = dot3(q0, uf), qsu = dot3(sv, uf);
#pragma unroll
  for (int k = 0; k < 3; ++k) { q0[k] -= q0u * uf[k]; qs[k] = sv[k] - qsu * uf[k]; }
  const float qa = dot3(qs, qs), qb = 2.f * dot3(q0, qs), qc = dot3(q0, q0) - rf * rf;
  const float disc = qb * qb - 4.f * qa * qc;
  const float sq = sqrtf(fmaxf(disc, 0.f)), i2a = 0.5f / fmaxf(qa, 1e-30f);
  const float lo = fmaxf(0.f, (-qb - sq) * i2a), hi = fminf(1.f, (-qb + sq) * i2a);
  const bool span = qa > 1e-12f && disc > 0.f && (hi - lo) * ls > 1e-3f;
  const float wg[3] = {sc.x[0] - r0[0], sc.x[1] - r0[1], sc.x[2] - r0[2]};
  const float tg = dot3(wg, sv) / (ls * ls);
  bool ok[2];
  float4 px[2];
#pragma unroll
  for (int e = 0; e < 2; ++e) {
    const float t = e ? hi : lo;
    float x[3], d[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) { x[k] = r0[k] + t * sv[k]; d[k] = x[k] - cf[k]; }
    const float g = dot3(d, uf), sep = g - 2.f * kCoreM;
    ok[e] = span && fabsf(t - tg) * ls > 1e-3f && sep < margin;
    px[e] = make_float4(x[0] - 0.5f * g * uf[0], x[1] - 0.5f * g * uf[1], x[2] - 0.5f * g * uf[2], sep);
  }
  // (quad-uniform: every input above is broadcast over the quad) with the GJK point alone the pair
  // falls through to the side-by-side test (quad_manifold), so nothing is written for it here
  if (write && (ok[0] || ok[1])) {
    if (j == 0) sink(0, make_float4(sc.x[0], sc.x[1], sc.x[2], sc.sep), sc.n);  // (GJK's normal: the warm start)
    if (j == 1 && ok[0]) sink(1, px[0], nr);
    if (j == 2 && ok[1]) sink(ok[0] ? 2 : 1, px[1], nr);
  }
  return 1 + (ok[0] ? 1 : 0) + (ok[1] ? 1 : 0);
}

// mode = cfg.self_manifold: 1 faces; 2 faces, else side-by-side rims; 3 faces, else a ruling on a
// face with at least one end point, else side-by-side rims (the oracle's self_manifold). kRf: mode 3 compiled in -- only the
// kernels launched for self_manifold 3 carry it (its code in the default kernel costs 0.9 % of the
// step through register allocation alone)
template <bool kRf, class Sink>
__device__ __forceinline__ int quad_manifold(const QCircle& h, int j, const SelfContact& sc, float margin, bool write,
                                             int mode, Sink sink) {
  const float sgd = (j & 2) ? 1.f : -1.f;
  const float dd[3] = {sgd * sc.n[0], sgd * sc.n[1], sgd * sc.n[2]};
  float u[3];
  cross3(h.e1, h.e2, u);
  const float iu = __builtin_amdgcn_rsqf(fmaxf(dot3(u, u), 1e-30f));
  u[0] *= iu; u[1] *= iu; u[2] *= iu;
  const float al = dot3(u, dd);
  const float r = sqrtf(dot3(h.e1, h.e1));
  const float sv = dot3(h.c, dd) + r * sqrtf(fmaxf(1.f - al * al, 0.f));
  const float psv = dppf<DPP_XOR1>(sv);
  const bool sup = (j & 1) ? (sv > psv) : !(psv > sv);
  int fm = (sup && fabsf(al) >= kFaceCos) ? (1 << j) : 0;
  fm |= dppi<DPP_XOR1>(fm);
  fm |= dppi<DPP_XOR2>(fm);
  const float so = al < 0.f ? -1.f : 1.f;
  const float uo[3] = {so * u[0], so * u[1], so * u[2]};
  if (!(fm & 3) || !(fm & 12)) {
    if (kRf && mode >= 3 && ((fm & 3) == 0) != ((fm & 12) == 0)) {  // a face on exactly one side
      const int k = quad_rimface(h, j, sc, margin, write, sink, fm, uo, r);
      if (k >= 2) return k;  // (the GJK point alone: the pair may still lie side by side)
    }
    return mode >= 2 ? quad_rim(h, j, sc, margin, write, sink) : 0;
  }
  const bool a1 = !(fm & 1), b3 = !(fm & 4);  // A's face on quad lane 1 (else 0), B's on 3 (else 2)
  float ca[3], ua[3], cb[3], ub[3];
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const float c0 = dppf<0x00>(h.c[k]), c1 = dppf<0x55>(h.c[k]), c2 = dppf<0xAA>(h.c[k]), c3 = dppf<0xFF>(h.c[k]);
    const float u0 = dppf<0x00>(uo[k]), u1 = dppf<0x55>(uo[k]), u2 = dppf<0xAA>(uo[k]), u3 = dppf<0xFF>(uo[k]);
    ca[k] = a1 ? c1 : c0; ua[k] = a1 ? u1 : u0;
    cb[k] = b3 ? c3 : c2; ub[k] = b3 ? u3 : u2;
  }
  const float r0 = dppf<0x00>(r), r1 = dppf<0x55>(r), r2 = dppf<0xAA>(r), r3 = dppf<0xFF>(r);
  const float ra = a1 ? r1 : r0, rb = b3 ? r3 : r2;
  const float nr[3] = {-ua[0], -ua[1], -ua[2]};  // the manifold's normal: A's face normal (B -> A)
  bool v[2];
  float4 px[2];  // this lane's two samples {x, sep}
#pragma unroll
  for (int side = 0; side < 2; ++side) {
    const float* cs = side ? ca : cb;
    const float* us = side ? ua : ub;
    const float* ct = side ? cb : ca;
    const float* ut = side ? ub : ua;
    const float rs = side ? ra : rb, rt = side ? rb : ra, sg = side ? -1.f : 1.f;
    float d0[3] = {ct[0] - cs[0], ct[1] - cs[1], ct[2] - cs[2]};
    const float du = dot3(d0, us);
    d0[0] -= du * us[0]; d0[1] -= du * us[1]; d0[2] -= du * us[2];
    const float dl = sqrtf(dot3(d0, d0));
    if (dl < 1e-9f) {  // concentric faces: a fixed in-plane axis
      const float ax[3] = {fabsf(us[0]) < 0.9f ? 1.f : 0.f, fabsf(us[0]) < 0.9f ? 0.f : 1.f, 0.f};
      const float au = dot3(ax, us);
      d0[0] = ax[0] - au * us[0]; d0[1] = ax[1] - au * us[1]; d0[2] = ax[2] - au * us[2];
      const float id0 = __builtin_amdgcn_rsqf(dot3(d0, d0));
      d0[0] *= id0; d0[1] *= id0; d0[2] *= id0;
    } else {
      const float id0 = 1.f / dl;
      d0[0] *= id0; d0[1] *= id0; d0[2] *= id0;
    }
    float d1[3];
    cross3(us, d0, d1);
    // this lane's sample j: (cr, sr) and whether the side has one
    float cr = 1.f, sr = 0.f;
    bool has;
    if (dl + rs <= rt) {
      has = true;
      cr = j == 0 ? 1.f : (j == 2 ? -1.f : 0.f);
      sr = j == 1 ? 1.f : (j == 3 ? -1.f : 0.f);
    } else if (dl + rt > rs) {
      const bool lens = dl < rs + rt;
      has = j == 0 || (lens && j < 3);
      if (j == 1 || j == 2) {
        const float c_ = clampf((dl * dl + rs * rs - rt * rt) / (2.f * dl * rs), -1.f, 1.f);
        const float s_ = sqrtf(fmaxf(1.f - c_ * c_, 0.f));
        cr = c_ * kFaceInsetC + s_ * kFaceInsetS;
        sr = (s_ * kFaceInsetC - c_ * kFaceInsetS) * (j == 1 ? 1.f : -1.f);
      }
    } else {
      has = false;
    }
    const float den = sg * dot3(nr, ut);
    float p[3], w[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) p[k] = cs[k] + rs * (cr * d0[k] + sr * d1[k]);
#pragma unroll
    for (int k = 0; k < 3; ++k) w[k] = ct[k] - p[k];
    const float t = dot3(w, ut) / (fabsf(den) < 1e-6f ? 1.f : den);
    float qv[3];
#pragma unroll
    for (int k = 0; k < 3; ++k) qv[k] = p[k] + t * sg * nr[k] - ct[k];
    const float sep = t - 2.f * kCoreM;
    v[side] = has && !(fabsf(den) < 1e-6f) && !(dot3(qv, qv) > rt * rt) && sep < margin;
    px[side] = make_float4(p[0] + 0.5f * t * sg * nr[0], p[1] + 0.5f * t * sg * nr[1], p[2] + 0.5f * t * sg * nr[2], sep);
  }
  int vm = (v[0] ? 1 << j : 0) | (v[1] ? 16 << j : 0);
  vm |= dppi<DPP_XOR1>(vm);
  vm |= dppi<DPP_XOR2>(vm);
  if (write) {
#pragma unroll
    for (int side = 0; side < 2; ++side) {
      const int k = __popc(vm & ((1 << (4 * side + j)) - 1));
      if (v[side] && k < 4) sink(k, px[side], nr);
    }
  }
  const int cnt = __popc(vm);
  return cnt < 4 ? cnt : 4;
}

// Detection + selection for the team's env; returns the number of contacts (team-uniform) and
// `over` (more than NCM candidates: slots go through MAP). Ground: lane s tests link s (the lowest
// rim point of each circle + 90-degree rotations, the first 4 within the margin). Self: a
// bounding-sphere broadphase (conservative, so it changes which pairs are tested, never which
// contacts are found), pairs split over the team; candidate pairs are split in rank order into
// contiguous chunks, one per lane, so candidates stay in canonical order lane by lane; each
// candidate pair runs GJK on the core hulls (gjk_pair, one contact per pair). Counting pass, team
// scan, then each lane writes its candidates at their canonical positions.
template <bool kRf>
__device__ __forceinline__ int detect(const zb_task_cfg& cfg, float Pz, const Q& q, bool warm, bool& over, Stamps& sp) {
  const float margin = cfg.contact_margin;

  // ground, counting pass: lane s = link s; keep the world circle frames for the write pass
  const int l = q.s < NL ? q.s : NL - 1;
  float C[2][3], E1[2][3], E2[2][3], cr0[2], sr0[2];
  unsigned vmask = 0;  // valid rim candidates (bit 4 ci + r), first 4 only
  {
    float R[9], p[3];
    read_frame(q, link_body(l), R, p);
    const float4* L = q.link(l);
    const float4 bd = L[0];
    float bc[3];
    mv3f(R, bd, bc);
    const bool near = q.s < NL && !(Pz + p[2] + bc[2] - bd.w > margin);
    int tk = 0;
#pragma unroll
    for (int ci = 0; ci < 2; ++ci) {
      const float4 cc = L[1 + 3 * ci];
      const bool face = cc.w == 0.f;  // not a duplicate of a lower link's mated face
      mv3f(R, cc, C[ci]);
      mv3f(R, L[2 + 3 * ci], E1[ci]);
      mv3f(R, L[3 + 3 * ci], E2[ci]);
      C[ci][0] += p[0]; C[ci][1] += p[1]; C[ci][2] += p[2];
      // lowest rim point, biased toward E1 so a flat disk gets a fixed body-attached manifold
      const float al = -E1[ci][2] + RIM_EPS, be = -E2[ci][2];
      const float nrm = sqrtf(al * al + be * be);
      cr0[ci] = 1.f; sr0[ci] = 0.f;
      if (nrm > 1e-12f) { cr0[ci] = al / nrm; sr0[ci] = be / nrm; }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float c0 = cr0[ci], s0 = sr0[ci];
        const float cr = r == 0 ? c0 : (r == 1 ? -s0 : (r == 2 ? -c0 : s0));
        const float sr = r == 0 ? s0 : (r == 1 ? c0 : (r == 2 ? -s0 : -c0));
        const float z = C[ci][2] + cr * E1[ci][2] + sr * E2[ci][2];
        if (near && face && Pz + z < margin && tk < 4) { vmask |= 1u << (4 * ci + r); ++tk; }
      }
    }
  }
  const int cnt_g = __popc(vmask);
  // ground candidates go first in canonical order: their positions follow from the ground counts
  // alone, so they are written now (the circle frames are dead before the self-collision pass)
  const int g_incl = tscan(cnt_g);
  const int g_tot = tbi<TL - 1>(g_incl);
  if (cnt_g) {
    int pos = g_incl - cnt_g;
    const float code = (float)(16 * l);
#pragma unroll
    for (int ci = 0; ci < 2; ++ci)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        if (vmask & (1u << (4 * ci + r))) {
          const float c0 = cr0[ci], s0 = sr0[ci];
          const float cr = r == 0 ? c0 : (r == 1 ? -s0 : (r == 2 ? -c0 : s0));
          const float sr = r == 0 ? s0 : (r == 1 ? c0 : (r == 2 ? -s0 : -c0));
          float x[3];
#pragma unroll
          for (int a = 0; a < 3; ++a) x[a] = C[ci][a] + cr * E1[ci][a] + sr * E2[ci][a];
          q.cand(pos, 0) = make_float4(x[0], x[1], x[2], Pz + x[2]);
          q.cand(pos, 1) = make_float4(0.f, 0.f, 1.f, code);
          ++pos;
        }
  }
  sp.mark(1);

  // self: broadphase (lane s: pairs [PAIRS_PER_LANE s, +PAIRS_PER_LANE)), team OR of the bits,
  // then the separating-axis test and GJK on the undecided pairs, dealt round-robin by rank over
  // the team. Pass 0 finds the contacts (and keeps each lane's first); the team OR of the contact
  // bits by rank gives every contact its canonical position (popcount of the lower ranks); pass 1
  // writes them, re-running GJK only for a lane's second and later contacts. One GJK call site.
  int s_tot = 0;
  if (cfg.enable_self_collision) {
    // lane l builds link l's world core hull once; its two circle centres + core radius are the
    // link's capsule (broadphase), the pair tests below gather the hulls with ds_bpermute
    Hull lh;
    world_hull(q, q.s < NL ? q.s : NL - 1, lh);
    if (q.s < NL) {
      const float rc = q.link(q.s)[2].w;
      q.cap(q.s, 0) = make_float4(lh.c[0][0], lh.c[0][1], lh.c[0][2], rc);
      q.cap(q.s, 1) = make_float4(lh.c[1][0], lh.c[1][1], lh.c[1][2], rc);
    }
    wave_sync();  // capsules
    // broadphase: capsule (segment of the core circle centres, radius = the larger core radius)
    // distance within margin + 2 kCoreM; conservative, so it changes which pairs are tested, never
    // which contacts are found (~13 of the 55 pairs pass on random-action rollouts: one round of
    // separating-axis tests instead of two with bounding spheres)
    unsigned long long mask = 0ull;
#pragma unroll
    for (int j = 0; j < PAIRS_PER_LANE; ++j) {
      const int pidx = PAIRS_PER_LANE * q.s + j;
      if (pidx < NPAIR) {
        const int code = q.pair_code(pidx);
        const float4 A0 = q.cap(code >> 4, 0), A1 = q.cap(code >> 4, 1);
        const float4 B0 = q.cap(code & 15, 0), B1 = q.cap(code & 15, 1);
        const float rr = A0.w + B0.w + margin + 2.f * kCoreM + 1e-5f;
        if (seg_seg_d2(A0, A1, B0, B1) <= rr * rr) mask |= 1ull << pidx;
      }
    }
    {
      const int lo = tor((int)(unsigned)mask), hi = tor((int)(unsigned)(mask >> 32));
      mask = (unsigned long long)(unsigned)lo | ((unsigned long long)(unsigned)hi << 32);
    }
    const int K = __popcll(mask);
    const int rounds = (K + TL - 1) / TL;
#ifdef ZB_STAMP_DETECT
    sp.mark(10);  // diagnostic split of the self-collision phase: broadphase
#endif
    // pair of rank r (r-th broadphase pair in index order) goes to lane r % TL: neighbouring pairs
    // of a folded robot, which tend to be in contact together, land on different lanes
    const unsigned long long bmask = mask;
    unsigned undecided = 0u;  // bit k: this lane's pair of round k needs GJK
    {
      // the pair tests gather both hulls from the link lanes with ds_bpermute (no per-pair frame
      // reads, link-table loads or rotations). The loop runs the wave's largest round count so
      // every lane takes part in each permute.
      const int rounds_w = max(max(__builtin_amdgcn_readlane(rounds, 0), __builtin_amdgcn_readlane(rounds, TL)),
                               max(__builtin_amdgcn_readlane(rounds, 2 * TL), __builtin_amdgcn_readlane(rounds, 3 * TL)));
      const int base = q.lane & ~(TL - 1);
      for (int k = 0; k < rounds_w; ++k) {
        const int r = q.s + TL * k;
        const bool valid = r < K;
        const int pcode = valid ? q.pair_code(nth_set_bit(bmask, r)) : 0x01;
        Hull A, B;
        gather_hull(lh, 4 * (base + (pcode >> 4)), A);
        gather_hull(lh, 4 * (base + (pcode & 15)), B);
        if (valid && !hulls_separated(A, B, margin + 2.f * kCoreM)) undecided |= 1u << k;
      }
    }
#ifdef ZB_STAMP_DETECT
    sp.mark(11);  // separating-axis tests
#endif
    // the undecided pairs of the whole team by rank; pair u runs GJK on quad u % 4 of the team in
    // round u / 4 (up to 4 pairs at once: random-action rollouts have at most 4 per env)
    unsigned long long und = 0ull;  // team: bit r = the pair of rank r needs GJK
    {
      unsigned long long mine = 0ull;
      for (int k = 0; k < rounds; ++k)
        if ((undecided >> k) & 1u) mine |= 1ull << (q.s + TL * k);
      const int lo = tor((int)(unsigned)mine), hi = tor((int)(unsigned)(mine >> 32));
      und = (unsigned long long)(unsigned)lo | ((unsigned long long)(unsigned)hi << 32);
    }
    const int U = __popcll(und);
    sp.note_pairs(U);
    const int qd = q.s >> 2, qj = q.s & 3;  // quad of the team, lane in the quad
    const int urounds = (U + 3) >> 2;
#ifdef ZB_STAMPS
    int deep_quad = 0;  // diagnostic: this quad's contacts on overlapping cores
#endif
    // this quad's first two contacts are kept for the write pass, which re-runs GJK only for a third
    // (round 6: the re-runs cost 3 % of the step at 4096 envs -- folded robots, whose quads hold two
    // contact pairs, are the slow waves; ZB_DIAG_NO_RERUN bounds it)
    SelfContact hit0 = {}, hit1 = {};
    int hit0_k = -1, hit1_k = -1;
    // bit k: this quad's pair of round k is a contact (own) of points - 1 = lo + 2 hi (own_lo / own_hi)
    unsigned own = 0u, own_lo = 0u, own_hi = 0u;
    // team, bit r: the pair of rank r is a contact (allhits), its points - 1 = exl + 2 exh: a pair's
    // first candidate position is g_tot + the points of the lower ranks
    unsigned long long allhits = 0ull, exl = 0ull, exh = 0ull;
    const bool mfon = cfg.self_manifold != 0;
#pragma unroll 1
    for (int pass = 0; pass < 2; ++pass) {
      for (int k = 0; k < urounds; ++k) {
        const int u = qd + 4 * k;
        if (u >= U) break;
        const int r = nth_set_bit(und, u);
        const unsigned long long lowr = (1ull << r) - 1ull;
        const int pos = g_tot + __popcll(allhits & lowr) + __popcll(exl & lowr) + 2 * __popcll(exh & lowr);
        const bool need = pass == 0 || (((own >> k) & 1u) != 0u && pos < g_tot + NSELF);
        if (!need) continue;
        const int pcode = q.pair_code(nth_set_bit(bmask, r));
        SelfContact sc = hit0;
        if (pass == 1 && k == hit1_k) {
          sc.n[0] = hit1.n[0]; sc.n[1] = hit1.n[1]; sc.n[2] = hit1.n[2];
          sc.x[0] = hit1.x[0]; sc.x[1] = hit1.x[1]; sc.x[2] = hit1.x[2];
          sc.sep = hit1.sep;
        }
        QCircle hc;
        quad_circle(q, (qj & 2) ? (pcode & 15) : (pcode >> 4), qj & 1, hc);
#ifdef ZB_DIAG_NO_RERUN  // diagnostic build (wrong contacts): what the write pass's GJK re-runs cost
        if (pass == 0) {
#else
        if (pass == 0 || (k != hit0_k && k != hit1_k)) {
#endif
          // start: the pair's contact normal of the previous substep of this step (kept contacts
          // hold {n, code} in FRC; unused slots code -1), else the hull centre difference
          float v0[3];
          {
            float ca[3], cb[3];
            quad_centres(hc, ca, cb);
            v0[0] = ca[0] - cb[0]; v0[1] = ca[1] - cb[1]; v0[2] = ca[2] - cb[2];
          }
          bool hot = false;  // warm start from a kept contact of the previous substep
          if (warm) {
            // (downwards: the pair's first kept point wins, the oracle's first match -- a rim
            // manifold's GJK point, whose GJK normal is the better start than its ends' normal)
#pragma unroll
            for (int c = NCM - 1; c >= 0; --c) {
              const float4 f = q.frc(c);
              const bool m = f.w == (float)(pcode + 1);
              v0[0] = m ? f.x : v0[0]; v0[1] = m ? f.y : v0[1]; v0[2] = m ? f.z : v0[2];
              hot = hot || m;
            }
          }
          int its = 0;
          const bool h = gjk_quad(hc, qj, v0, hot, pass == 0 ? margin : 1e30f, pass == 0 ? margin : 1e30f, sc, its);
          if (qj == 0) {
            sp.count(kStampCount0, 1);
            sp.count(kStampCount0 + 1, its);
          }
          sp.note_its(its);
          if (pass == 0 && h) {
            if (own == 0u) {
              hit0 = sc;
              hit0_k = k;
            } else if (hit1_k < 0) {
              hit1 = sc;
              hit1_k = k;
            }
            own |= 1u << k;
#ifdef ZB_STAMPS
            if (qj == 0 && sc.sep <= -2.f * kCoreM + 1e-7f) ++deep_quad;
#endif
          }
          if (pass == 0 && !h) continue;
        }
        // the face manifold of a contact (cores apart: the overlap estimate stays one point); the
        // write pass stores its points
        const float code = (float)(pcode + 1);
        const int mc = (mfon && sc.sep > -2.f * kCoreM + 1e-7f)
                           ? quad_manifold<kRf>(hc, qj, sc, margin, pass == 1, cfg.self_manifold, [&](int rank, float4 xs, const float* nn) {
                               if (pos + rank < g_tot + NSELF) {
                                 q.cand(pos + rank, 0) = xs;
                                 q.cand(pos + rank, 1) = make_float4(nn[0], nn[1], nn[2], code);
                               }
                             })
                           : 0;
        if (pass == 0) {
          own_lo |= (mc == 2 || mc == 4) ? 1u << k : 0u;
          own_hi |= mc >= 3 ? 1u << k : 0u;
        } else if (mc == 0 && qj == 0) {
          q.cand(pos, 0) = make_float4(sc.x[0], sc.x[1], sc.x[2], sc.sep);
          q.cand(pos, 1) = make_float4(sc.n[0], sc.n[1], sc.n[2], (float)(pcode + 1));
        }
      }
      if (pass == 0) {  // the team's contacts by rank: canonical positions follow the ground ones
        unsigned long long m1 = 0ull, ml = 0ull, mh = 0ull;
        for (int k = 0; k < urounds; ++k) {
          const int u = qd + 4 * k;
          if (u < U && ((own >> k) & 1u)) {
            const unsigned long long bit = 1ull << nth_set_bit(und, u);
            m1 |= bit;
            ml |= ((own_lo >> k) & 1u) ? bit : 0ull;
            mh |= ((own_hi >> k) & 1u) ? bit : 0ull;
          }
        }
        auto team_or = [](unsigned long long m) {
          const int lo = tor((int)(unsigned)m), hi = tor((int)(unsigned)(m >> 32));
          return (unsigned long long)(unsigned)lo | ((unsigned long long)(unsigned)hi << 32);
        };
        allhits = team_or(m1);
        exl = team_or(ml);
        exh = team_or(mh);
        s_tot = __popcll(allhits) + __popcll(exl) + 2 * __popcll(exh);
      }
    }
#ifdef ZB_STAMPS
    {
      const int deep = (int)tsum((float)deep_quad);
      if (q.s == 0) sp.note_caps(g_tot, s_tot, deep);
    }
#endif
  }
#ifdef ZB_STAMPS
  else if (q.s == 0) sp.note_caps(g_tot, 0, 0);
#endif
  sp.mark(2);
  const int n = g_tot + min(s_tot, NSELF);
  over = n > NCM;

  // overflow (rare): rank every candidate by (sep, canonical index); MAP = kept positions in order
  if (__ballot(over) != 0ull) {
    wave_sync();
    if (over)
      for (int p = q.s; p < n; p += TL) {
        const float sp_ = q.cand(p, 0).w;
        int r = 0;
        for (int j = 0; j < n; ++j) {
          const float sj = q.cand(j, 0).w;
          r += (sj < sp_ || (sj == sp_ && j < p)) ? 1 : 0;
        }
        q.keep(p) = r < NCM ? 1 : 0;
      }
    wave_sync();
    if (over && q.s < NCM) {
      int c = 0, pos = -1;
      for (int p = 0; p < n; ++p)
        if (q.keep(p) != 0) {
          if (c == q.s) pos = p;
          ++c;
        }
      q.map(q.s) = pos;
    }
  }
  wave_sync();
  return over ? NCM : n;
}

__device__ __forceinline__ void tangents(const float n[3], float t1[3], float t2[3]) {
  if (fabsf(n[2]) < 0.9f) {
    const float s = sqrtf(n[1] * n[1] + n[0] * n[0]);
    t1[0] = -n[1] / s; t1[1] = n[0] / s; t1[2] = 0.f;
  } else {
    const float s = sqrtf(n[2] * n[2] + n[1] * n[1]);
    t1[0] = 0.f; t1[1] = n[2] / s; t1[2] = -n[1] / s;
  }
  cross3(n, t1, t2);
}

// What the MDP needs from a substep (instead of 12 per-link force vectors).
struct SensorOut {
  float feet_f[2][3];   // net contact force on foot_0 / foot_1
  float undes_fmax;     // max over the 10 undesired links of |net force|
  float tau2;           // sum of squared Isaac Lab applied torques (torques reward)
};

// Isaac Lab's ContactSensor with history_length > 0 updates after every physics step
// (SensorBase.update -> _update_outdated_buffers on each scene.update(physics_dt)): each substep
// parks its sensor record in LDS (one lane per env), the MDP epilogue replays them.
__device__ __forceinline__ void sens_record(const Q& q, int k, const SensorOut& so) {
  if (q.s == 0) {
    q.sens(k, 0) = make_float4(so.feet_f[0][2], so.feet_f[1][2], sqrtf(dot3(so.feet_f[0], so.feet_f[0])),
                               sqrtf(dot3(so.feet_f[1], so.feet_f[1])));
    q.sens(k, 1) = make_float4(so.undes_fmax, 0.f, 0.f, 0.f);
  }
}

// After this step's `dec` physics steps: the sum of the feet F_z and the max undesired |F| over the
// HIST-slot histories (slot 0 newest; the slots older than this step come from the state rows
// fz_row / fm_row), and the air / contact timers advanced by dt per physics step
// (ContactSensor._update_buffers_impl: first contact -> last_air_time, first detach ->
// last_contact_time). Only reductions are kept in registers; sens_store writes the histories.
template <int HIST>
__device__ __forceinline__ void sens_replay(const Q& q, const float* __restrict__ st, int N, int i, int fz_row,
                                            int fm_row, int dec, float dt, float thr, float fz_sum[2], float& fm_max,
                                            float air_cur[2], float air_last[2], float con_cur[2], float con_last[2]) {
  fz_sum[0] = fz_sum[1] = 0.f;
  fm_max = 0.f;
#pragma unroll
  for (int h = 0; h < HIST; ++h) {
    float a0, a1, m;
    if (h < dec) {
      const float4 a = q.sens(dec - 1 - h, 0);
      a0 = a.x;
      a1 = a.y;
      m = q.sens(dec - 1 - h, 1).x;
    } else {
      const int j = h - dec;
      a0 = st[(size_t)(fz_row + 2 * j) * N + i];
      a1 = st[(size_t)(fz_row + 2 * j + 1) * N + i];
      m = st[(size_t)(fm_row + j) * N + i];
    }
    fz_sum[0] += a0;
    fz_sum[1] += a1;
    fm_max = h == 0 ? m : fmaxf(fm_max, m);
  }
  for (int k = 0; k < dec; ++k) {
    const float4 a = q.sens(k, 0);
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const bool c = (f == 0 ? a.z : a.w) > thr;
      air_last[f] = (air_cur[f] > 0.f && c) ? air_cur[f] + dt : air_last[f];
      air_cur[f] = c ? 0.f : air_cur[f] + dt;
      con_last[f] = (con_cur[f] > 0.f && !c) ? con_cur[f] + dt : con_last[f];
      con_cur[f] = c ? con_cur[f] + dt : 0.f;
    }
  }
}

// the new histories into the state rows (oldest slot first, so the carried slots are read before
// they are overwritten); zero = the env was reset (ContactSensor.reset)
template <int HIST, class Put>
__device__ __forceinline__ void sens_store(const Q& q, const float* __restrict__ st, int N, int i, int fz_row,
                                           int fm_row, int dec, bool zero, Put&& put) {
#pragma unroll
  for (int h = HIST - 1; h >= 0; --h) {
    float a0, a1, m;
    if (h < dec) {
      const float4 a = q.sens(dec - 1 - h, 0);
      a0 = a.x;
      a1 = a.y;
      m = q.sens(dec - 1 - h, 1).x;
    } else {
      const int j = h - dec;
      a0 = st[(size_t)(fz_row + 2 * j) * N + i];
      a1 = st[(size_t)(fz_row + 2 * j + 1) * N + i];
      m = st[(size_t)(fm_row + j) * N + i];
    }
    put(fz_row + 2 * h, zero ? 0.f : a0);
    put(fz_row + 2 * h + 1, zero ? 0.f : a1);
    put(fm_row + h, zero ? 0.f : m);
  }
}
template <int HIST>
__device__ __forceinline__ void sens_store(const Q& q, float* __restrict__ st, int N, int i, int fz_row, int fm_row,
                                           int dec, bool zero) {
  sens_store<HIST>(q, st, N, i, fz_row, fm_row, dec, zero,
                   [&](int row, float v) { st[(size_t)row * N + i] = v; });
}

// Staged epilogue: the writer lane of each env puts its outputs (state rows, then the observation,
// reward, terminated, truncated) into LDS (aliasing the contact rows, dead after the physics), and
// the whole wave stores them: one store instruction covers 16 state rows x the EPW consecutive
// envs of the workgroup, the EPW observation rows go out as one contiguous run. This replaces ~110
// single-lane-per-env store instructions per wave with ~9 full-wave ones.
__device__ __forceinline__ float& Q::stg(int k) const { return reinterpret_cast<float*>(b + YG_OFF)[e * STG_LEN + k]; }
template <int SD, int OD>
__device__ __forceinline__ void staged_store(const Q& q, int env0, int N, float* __restrict__ st,
                                             float* __restrict__ obs, float* __restrict__ rew,
                                             uint8_t* __restrict__ term, uint8_t* __restrict__ trunc,
                                             int64_t* __restrict__ done) {
  static_assert(SD + OD + 3 <= STG_LEN, "staging row");
  wave_sync();
  const float* S = reinterpret_cast<const float*>(q.b + YG_OFF);
  const int e = q.lane % EPW, f0 = q.lane / EPW;
  const int env = env0 + e;
  if (env < N) {
#pragma unroll
    for (int f = f0; f < SD; f += WGT / EPW) st[(size_t)f * N + env] = S[e * STG_LEN + f];
    if (f0 == 0) rew[env] = S[e * STG_LEN + SD + OD];
    if (f0 == 1) term[env] = S[e * STG_LEN + SD + OD + 1] != 0.f ? 1 : 0;
    if (f0 == 2) trunc[env] = S[e * STG_LEN + SD + OD + 2] != 0.f ? 1 : 0;
    // the caller's done buffer (zb_set_done_buffer): terminated | truncated as int64, rsl_rl's dones
    if (done && f0 == 3) done[env] = (S[e * STG_LEN + SD + OD + 1] != 0.f || S[e * STG_LEN + SD + OD + 2] != 0.f) ? 1 : 0;
  }
  const int nv = min(EPW, N - env0);
#pragma unroll
  for (int t = q.lane; t < EPW * OD; t += WGT)
    if (t < nv * OD) {
      obs[(size_t)env0 * OD + t] = S[(t / OD) * STG_LEN + SD + t % OD];
    }
}

// MDP carry prefetch: the env's MDP state rows (everything after the 25 physics rows) are loaded
// in the prologue, in the same batch as the physics rows, and parked in LDS across the substeps:
// lane s of team e loads rows CARRY0 + s + 16 k of env e, so one load instruction covers 16 rows x
// the EPW envs of the wave. The epilogue then reads LDS instead of waiting on ~40 HBM loads issued
// after the physics. Returns the env's carry row indexed by state row (valid for rows >= CARRY0).
template <int SD>
__device__ __forceinline__ const float* carry_prefetch(const Q& q, const float* __restrict__ st, int N, int i) {
  static_assert(SD - CARRY0 <= CARRY_W, "carry width");
  constexpr int K = (SD - CARRY0 + TL - 1) / TL;
  float v[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int r = CARRY0 + q.s + TL * k;
    v[k] = r < SD ? st[(size_t)r * N + i] : 0.f;
  }
  float* c = q.carry();
#pragma unroll
  for (int k = 0; k < K; ++k) c[q.s + TL * k] = v[k];
  return c - CARRY0;
}

// One Gauss-Seidel contact update (normal + Coulomb disk). g = {Y0[d], Y1[d], Y2[d], -} of this
// lane's coordinate d, a0 = {invm0, invm1, invm2, vmin invm0}, a1 = {c01 invm1, c02 invm2, -, -}
// (c0r = Y_r . Y_0), lam = {ln, l1, l2, broken}; mu / mu_d the static / dynamic coefficients. The three row dots are reduced across the team; the
// tangent velocities see the normal update through the cross terms. Arranged for a short
// dependency chain: the impulse-independent parts are formed while the normal row resolves, and
// the disk projection is min(1, lim / max(|l|, 1e-15)) (rsq; finite for |l| = 0). Returns the
// new impulses; wd (the lane's coordinate) updated.
__device__ __forceinline__ float4 pgs_update(const float4 g, const float4 a0, const float4 a1, const float4 lam,
                                             float mu, float mu_d, float& wd) {
  const float p0 = tsum(g.x * wd);
  const float p1 = tsum(g.y * wd);
  const float p2 = tsum(g.z * wd);
  const float ln = fmaxf(fmaf(-p0, a0.x, lam.x + a0.w), 0.f);
  const float dl = ln - lam.x;
  const float u1 = fmaf(-p1, a0.y, lam.y), u2 = fmaf(-p2, a0.z, lam.z);
  float l1 = fmaf(-a1.x, dl, u1);
  float l2 = fmaf(-a1.y, dl, u2);
  // static / dynamic Coulomb disk (PhysX's patch friction): the contact sticks while |l| <= mu ln;
  // once a loaded contact (ln > 0) exceeds the static cone it is "broken" (lam.w = 1) for the rest
  // of the substep's sweeps and slides with |l| = mu_d ln (mu_d = mu: the plain projection
  // min(1, mu ln / |l|)); an unloaded contact's friction is 0 without breaking it
  const float ri = __builtin_amdgcn_rsqf(fmaxf(fmaf(l1, l1, l2 * l2), 1e-30f));
  const float ts = mu * ln * ri, td = mu_d * ln * ri;  // the static / dynamic cone over |l|
  const bool over = ts < 1.f;
  const bool brk = (lam.w != 0.f) | (over & (ln > 0.f));  // (bitwise: no short-circuit branch)
  // (one select, no branch: unbroken, min(ts, 1) is ts inside the static cone and 1 outside it)
  const float sc = fminf(brk ? td : ts, 1.f);
  l1 *= sc;
  l2 *= sc;
  const float d1 = l1 - lam.y, d2 = l2 - lam.z;
  wd = fmaf(g.x, dl, wd);
  wd = fmaf(g.y, d1, wd);
  wd = fmaf(g.z, d2, wd);
  return make_float4(ln, l1, l2, brk ? 1.f : 0.f);
}

// mass-matrix column of joint K (computed in lane K) into every lane's packed lower triangle
template <int K>
__device__ __forceinline__ void crba_column(float L[NT], const float Fk[6], const float Mk[ND], float arm) {
#pragma unroll
  for (int a = 0; a < 6; ++a) L[tri(6 + K, a)] = tb<K>(Fk[a]);
#pragma unroll
  for (int jj = 0; jj <= K; ++jj) L[tri(6 + K, 6 + jj)] = tb<K>(Mk[jj]) + (jj == K ? arm : 0.f);
}

// Team-parallel Cholesky of the 12x12 mass matrix. Lane s owns row own_row(s) of M (joint rows
// 6 + s in lanes 0-5, where the CRBA leaves column s; root rows s - 6 in lanes 6-11) in R[].
// Column k: every lane forms its row's t = M[r][k] - sum_{m<k} L[r][m] L[k][m] (row k of L from
// its packed copy), the owner of row k broadcasts its t (the pivot), every lane takes
// iv = rsq(pivot) and scales, and column k (rows >= k) is broadcast from the row owners into every
// lane's packed L. ~200 instructions instead of the ~380 of the redundant factorisation; every
// lane ends with the full L / inv (lanes 12-15 own no row).
constexpr int own_lane(int r) { return r < 6 ? r + 6 : r - 6; }
template <int K, int Rw>
__device__ __forceinline__ void team_chol_bcast(float v, float L[NT]) {  // column K, rows Rw.. of L
  L[tri(Rw, K)] = tb<own_lane(Rw)>(v);
  if constexpr (Rw + 1 < NV) team_chol_bcast<K, Rw + 1>(v, L);
}
template <int K>
__device__ __forceinline__ void team_chol_col(float R[NV], float L[NT], float inv[NV]) {
  float t = R[K];
#pragma unroll
  for (int m = 0; m < K; ++m) t = fmaf(-R[m], L[tri(K, m)], t);
  const float pv = fmaxf(tb<own_lane(K)>(t), 1e-12f);
#if ZB_RSQ_NR
  // v_rsq_f32 (1 ulp) refined by one Newton step: every whitened quantity (the free velocity, the
  // contact rows Y = L^-1 J^T, their effective masses) is scaled by these pivots
  float iv = __builtin_amdgcn_rsqf(pv);
  iv = fmaf(0.5f * iv, fmaf(-pv * iv, iv, 1.f), iv);
#else
  const float iv = __builtin_amdgcn_rsqf(pv);
#endif
  inv[K] = iv;
  R[K] = t * iv;
  L[tri(K, K)] = pv * iv;
  if constexpr (K + 1 < NV) team_chol_bcast<K, K + 1>(R[K], L);
}
__device__ __forceinline__ void cholesky_team(float R[NV], float L[NT], float inv[NV]) {
  team_chol_col<0>(R, L, inv); team_chol_col<1>(R, L, inv); team_chol_col<2>(R, L, inv);
  team_chol_col<3>(R, L, inv); team_chol_col<4>(R, L, inv); team_chol_col<5>(R, L, inv);
  team_chol_col<6>(R, L, inv); team_chol_col<7>(R, L, inv); team_chol_col<8>(R, L, inv);
  team_chol_col<9>(R, L, inv); team_chol_col<10>(R, L, inv); team_chol_col<11>(R, L, inv);
}
// x[s] in lanes s < N (a lane-dependent index into a team-uniform array), 0 in the others
template <int N>
__device__ __forceinline__ float pick_lane(const float (&x)[N], int s) {
  float v = 0.f;
#pragma unroll
  for (int j = 0; j < N; ++j) v = s == j ? x[j] : v;
  return v;
}
// Team forward substitution z = L^-1 y, columns K..KE-1. Lane s owns row r = own_row(s) with its
// L row in R (cholesky_team) and t = y_r - sum_{k<K} L[r][k] z_k; z_K = t_owner / L_KK is
// broadcast from the owner of row K, every lane removes its row's z_K term, and the owner keeps
// z_K in wd. Lanes past their own row carry a meaningless t.
template <int K, int KE>
__device__ __forceinline__ void team_fwd(const float R[NV], const float inv[NV], float& t, float z[NV], float& wd,
                                         int s) {
  const float zk = tb<own_lane(K)>(t) * inv[K];
  z[K] = zk;
  wd = s == own_lane(K) ? zk : wd;
  t = fmaf(-R[K], zk, t);
  if constexpr (K + 1 < KE) team_fwd<K + 1, KE>(R, inv, t, z, wd, s);
}

// contact bias velocity: a speculative contact (sep >= 0) may close its gap within the step h it
// is solved for (PGS: the substep dt; TGS: the sub-iteration dt / iterations); a penetration is
// pushed out at baumgarte * depth per substep, capped at max_depenetration_velocity
// (zbot_cfg.py:633). Same as the oracle's contact_bias.
__device__ __forceinline__ float contact_bias(const zb_task_cfg& cfg, MP m, float sep, float h, float dt) {
  // (both sides evaluated and selected: no divergent branch in the TGS sub-iterations)
  const float spec = -sep / h, push = fminf(cfg.baumgarte * (-sep) / dt, m->max_depenetration_velocity);
  return sep >= 0.f ? spec : push;
}
// joint speed clamp (actuator velocity_limit) and root link angular speed limit (rigid props
// max_angular_velocity; PhysX scales the vector)
__device__ __forceinline__ void clamp_speeds(MP m, float u[NV]) {
#pragma unroll
  for (int j = 0; j < ND; ++j) u[6 + j] = clampf(u[6 + j], -m->velocity_limit, m->velocity_limit);
  const float w2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
  const float wmax = m->max_angular_velocity;
  const float sc = w2 > wmax * wmax ? wmax * __builtin_amdgcn_rsqf(w2) : 1.f;
  u[0] *= sc; u[1] *= sc; u[2] *= sc;
}

// ground rim candidate r (0: the lowest rim point, 1-3: its 90-degree rotations) of circle ci of
// link l at the pose in LDS, relative to that pose's root origin: detect's formula (oracle
// ground_rim_point). Used by the TGS refresh (kRefresh).
__device__ __forceinline__ void ground_rim_point(const Q& q, int l, int ci, int r, float x[3]) {
  float R[9], p[3];
  read_frame(q, link_body(l), R, p);
  const float4* L = q.link(l);
  float C[3], E1[3], E2[3];
  mv3f(R, L[1 + 3 * ci], C);
  mv3f(R, L[2 + 3 * ci], E1);
  mv3f(R, L[3 + 3 * ci], E2);
  C[0] += p[0]; C[1] += p[1]; C[2] += p[2];
  const float al = -E1[2] + RIM_EPS, be = -E2[2];
  const float nrm = sqrtf(al * al + be * be);
  float c0 = 1.f, s0 = 0.f;
  if (nrm > 1e-12f) { c0 = al / nrm; s0 = be / nrm; }
  const float cr = r == 0 ? c0 : (r == 1 ? -s0 : (r == 2 ? -c0 : s0));
  const float sr = r == 0 ? s0 : (r == 1 ? c0 : (r == 2 ? -s0 : -c0));
#pragma unroll
  for (int a = 0; a < 3; ++a) x[a] = C[a] + cr * E1[a] + sr * E2[a];
}

// the pose integration of a substep over time T with the pose velocity ua (root twist at P) and
// wv = omega x v_P at the substep start (oracle advance_pose): root origin += T (v + T wv), the
// orientation by the exact exponential map, joints += T qdot wrapped as PhysX reports them
__device__ __forceinline__ void advance_pose(Phys& s, const float ua[NV], const float wv[3], float T) {
#pragma unroll
  for (int a = 0; a < 3; ++a) s.pos[a] += T * (ua[3 + a] + T * wv[a]);
  {
    const float th = sqrtf(ua[0] * ua[0] + ua[1] * ua[1] + ua[2] * ua[2]) * T;
    float dq[4];
    if (th > 1e-12f) {
      float sn, cs;
      sincos_r(0.5f * th, &sn, &cs);
      const float sc = sn / th * T;
      dq[0] = cs; dq[1] = ua[0] * sc; dq[2] = ua[1] * sc; dq[3] = ua[2] * sc;
    } else {
      dq[0] = 1.f; dq[1] = 0.5f * T * ua[0]; dq[2] = 0.5f * T * ua[1]; dq[3] = 0.5f * T * ua[2];
    }
    float qn[4];
    qmul(dq, s.quat, qn);
    qnormalize(qn);
    s.quat[0] = qn[0]; s.quat[1] = qn[1]; s.quat[2] = qn[2]; s.quat[3] = qn[3];
  }
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    float qv = s.jq[j] + T * ua[6 + j];
    if (qv > TWO_PI_F) qv -= 2.f * TWO_PI_F;
    else if (qv < -TWO_PI_F) qv += 2.f * TWO_PI_F;
    s.jq[j] = qv;
  }
}

// TGS per-position-iteration refresh of the ground contacts (solver_modes 2, 3; oracle substep,
// `refresh`): the pose after T = it h with the mean velocity of the sub-iterations so far
// (wm = this lane's coordinate of the mean w; the same integration as the substep's end), FK
// there, and lane c re-evaluates its ground contact: the rim candidate re-supported at that pose,
// the separation, the three Jacobian rows (the root columns still at the substep's P, the mass
// matrix factor the substep's), the effective masses, cross terms and bias. Self contacts keep the
// linear advance in mode 2 and are refreshed in mode 3 (below). The LDS pose records hold the refreshed pose afterwards (nothing later in the
// substep reads them; the next substep's FK rewrites them).
__device__ __forceinline__ void refresh_contacts(const zb_task_cfg& cfg, MP m, const Phys& s, const Q& q, const float L[NT],
                                              const float Li[NV], float wm, float T, float hsub, float dt, int nc,
                                              int rim_own, int gl_own, const float anc[6], float& sep_own) {
  float w[NV], um[NV];
  w[0] = tb<own_lane(0)>(wm); w[1] = tb<own_lane(1)>(wm); w[2] = tb<own_lane(2)>(wm);
  w[3] = tb<own_lane(3)>(wm); w[4] = tb<own_lane(4)>(wm); w[5] = tb<own_lane(5)>(wm);
  w[6] = tb<own_lane(6)>(wm); w[7] = tb<own_lane(7)>(wm); w[8] = tb<own_lane(8)>(wm);
  w[9] = tb<own_lane(9)>(wm); w[10] = tb<own_lane(10)>(wm); w[11] = tb<own_lane(11)>(wm);
  bwd_sub(L, Li, w, um);
  clamp_speeds(m, um);
  float wv[3];
  cross3(s.av, s.lv, wv);
  Phys p2 = s;
  advance_pose(p2, um, wv, T);
  wave_sync();
  fk_team_pose(p2, q);
  wave_sync();
  // self contacts (solver_mode 3): lane c's body-fixed anchors anc (pa on A, pb on B, placed at the
  // substep's pose so that n.(pa - pb) is the detected separation) carried to the advanced pose; the
  // separation n.(pa' - pb') along the substep's normal, the rows at the anchors' midpoint
  const bool self_ref = cfg.solver_mode == 3 && rim_own < 0;
  if (q.s < nc && (rim_own >= 0 || self_ref)) {
    const int c = q.s;
    const float4 fr = q.frc(c);  // the substep's normal and code
    const int code = (int)fr.w;
    const int lb = (code & 15) - 1;
    const bool gnd = rim_own >= 0;
    const int ba = link_body(gnd ? gl_own : code >> 4), bb = gnd ? -1 : link_body(lb);
    float x[3], sep, n[3];
    if (gnd) {
      ground_rim_point(q, gl_own, rim_own >> 2, rim_own & 3, x);
      sep = p2.pos[2] + x[2];
      n[0] = 0.f; n[1] = 0.f; n[2] = 1.f;
    } else {
      float R[9], pA[3], pB[3], pa[3], pb[3];
      read_frame(q, ba, R, pA);
      mv3(R, anc, pa);
      read_frame(q, bb, R, pB);
      mv3(R, anc + 3, pb);
#pragma unroll
      for (int a = 0; a < 3; ++a) { pa[a] += pA[a]; pb[a] += pB[a]; }
      n[0] = fr.x; n[1] = fr.y; n[2] = fr.z;
      sep = n[0] * (pa[0] - pb[0]) + n[1] * (pa[1] - pb[1]) + n[2] * (pa[2] - pb[2]);
#pragma unroll
      for (int a = 0; a < 3; ++a) x[a] = 0.5f * (pa[a] + pb[a]);
    }
    const float root = gnd ? 1.f : 0.f;  // self contacts: the root terms cancel
    const float xr[3] = {x[0] + (p2.pos[0] - s.pos[0]), x[1] + (p2.pos[1] - s.pos[1]), x[2] + (p2.pos[2] - s.pos[2])};
    float S[ND][6], org[ND][3];
    read_joints(q, S, org);
    float cj[ND][3];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float xo[3] = {x[0] - org[j][0], x[1] - org[j][1], x[2] - org[j][2]};
      float c3[3];
      cross3(S[j], xo, c3);
      const float sg = (j < ba ? 1.f : 0.f) - (j < bb ? 1.f : 0.f);
      cj[j][0] = sg * c3[0]; cj[j][1] = sg * c3[1]; cj[j][2] = sg * c3[2];
    }
    float t1[3], t2[3];
    tangents(n, t1, t2);
    float invm[3], Y[3][NV];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      float d[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) d[a] = r == 0 ? n[a] : (r == 1 ? t1[a] : t2[a]);
      float J[NV], xd[3];
      cross3(xr, d, xd);
      J[0] = root * xd[0]; J[1] = root * xd[1]; J[2] = root * xd[2];
      J[3] = root * d[0]; J[4] = root * d[1]; J[5] = root * d[2];
#pragma unroll
      for (int j = 0; j < ND; ++j) J[6 + j] = dot3(cj[j], d);
      fwd_sub(L, Li, J, Y[r]);
      invm[r] = 1.f / (dot12(Y[r], Y[r]) + 1e-9f);
    }
#pragma unroll
    for (int d = 0; d < NV; ++d) q.yg_at(c, own_lane(d)) = make_float4(Y[0][d], Y[1][d], Y[2][d], 0.f);
    sep_own = sep;
    const float4 a1 = q.aux(c, 1);
    q.aux(c, 0) = make_float4(invm[0], invm[1], invm[2], contact_bias(cfg, m, sep, hsub, dt) * invm[0]);
    q.aux(c, 1) = make_float4(dot12(Y[1], Y[0]) * invm[1], dot12(Y[2], Y[0]) * invm[2], a1.z, a1.w);
  }
  wave_sync();
}

// ------------------------------------------------------------------------- one substep
// kLinkFriction: per-contact Coulomb coefficient from the per-link table q.fric (standup DR);
// otherwise cfg.friction everywhere.
// kRefresh (zb_task_cfg.solver_mode 2 / 3, with kTgs): before every sub-iteration after the first the
// ground contacts (mode 3: and the self contacts) are re-evaluated at the pose the sub-iterations so far reached (see the sweeps).
template <bool kDebugForces, bool kLinkFriction, bool kTgs, bool kRefresh = false, bool kRf = false>
__device__ __forceinline__ void substep(MP m0, const zb_task_cfg& cfg, Phys& s,
                                        const float target[ND], const Q& q, bool last, bool warm, SensorOut& so,
                                        float (*dbgF)[3], float* dbgTau, Stamps& sp) {
  // (dt through an empty asm: its own scalar register, not a lane of the cfg words the compiler
  // loads as one 16-register tuple, which a spill would reload whole at every use)
  float dt = cfg.sim_dt;
  asm volatile("" : "+s"(dt));
  MP m = opaque(m0);

  if (last) {
    float t2 = 0.f;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float t = clampf(m->kp * (target[j] - s.jq[j]) - m->kd * s.jqd[j], -m->effort_limit, m->effort_limit);
      t2 += t * t;
      if (kDebugForces) dbgTau[j] = t;
    }
    so.tau2 = t2;
  }

  SI Ib;                   // this lane's body (b = s < NB; zero elsewhere)
  float Sown[6];           // this lane's joint motion subspace (j = s < ND; zero elsewhere)
  int nc;
  bool over;
  wave_sync();  // the previous substep's LDS readers are done
  fk_team<true>(s, q, Ib, Sown);
  wave_sync();
  sp.mark(9);
  nc = detect<kRf>(cfg, s.pos[2], q, warm, over, sp);
  m = opaque(m0);

  // RNEA bias forces (qddot = 0, gravity as base acceleration) and, in the same team suffix sum,
  // the generalised momentum: lane b runs the velocity / acceleration chain up to its body
  // (joints j >= b contribute zero) and forms g_b = I_b V_b - dt f_b; the suffix sum
  // G_b = sum_{b' >= b} g_b' (DPP row shifts) gives the implicit velocity update's right-hand side
  // M u - dt C row by row: root rows G_0 (lane 0's sum), joint row j S_j . G_{j+1} (lane j). Each
  // lane keeps the entry of the row it owns in the team Cholesky (own_row), so the free velocity
  // needs one team forward substitution instead of L^T u plus a redundant L^-1 b.
  const float arm = dt * (m->kd + dt * m->kp);
  float L[NT];
  float R[NV];   // this lane's row of M (cholesky_team)
  float yown;    // this lane's row of M u - dt C
  {
  float S[ND][6];  // joint motion subspaces (LDS), live through RNEA + CRBA only
  read_S(q, S);
  {
    const int b = q.s;
    float V[6] = {s.av[0], s.av[1], s.av[2], s.lv[0], s.lv[1], s.lv[2]};
    float A[6] = {0.f, 0.f, 0.f, 0.f, 0.f, cfg.gravity};
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float qd = j < b ? s.jqd[j] : 0.f;
#pragma unroll
      for (int a = 0; a < 6; ++a) V[a] += S[j][a] * qd;
      float t1[3], t2[3], t3[3];
      cross3(V, S[j], t1);
      cross3(V, S[j] + 3, t2);
      cross3(V + 3, S[j], t3);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        A[a] += t1[a] * qd;
        A[3 + a] += (t2[a] + t3[a]) * qd;
      }
    }
    float g[6];
    {
      float IA[6], IV[6], t1[3], t2[3], t3[3];
      si_mul(Ib, A, IA);
      si_mul(Ib, V, IV);
      cross3(V, IV, t1);
      cross3(V + 3, IV + 3, t2);
      cross3(V, IV + 3, t3);
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        g[a] = fmaf(-dt, IA[a] + t1[a] + t2[a], IV[a]);
        g[3 + a] = fmaf(-dt, IA[3 + a] + t3[a], IV[3 + a]);
      }
    }
    suffix_sum<6>(g);
    float yj = 0.f, yr = 0.f;
    const int r = q.s - 6;  // root row of lanes 6-11
#pragma unroll
    for (int a = 0; a < 6; ++a) {
      yj = fmaf(Sown[a], dppzf<DPP_SHL + 1>(g[a]), yj);  // G_{j+1} in lane j
      const float g0 = tb<0>(g[a]);
      yr = r == a ? g0 : yr;
    }
    yown = q.s < ND ? yj : yr;  // lanes 12-15: 0
  }

  // CRBA: composite inertias by a team suffix sum; lane k forms F_k = Ic_{k+1} S_k and its
  // mass-matrix column S_jj . F_k, then the team assembles the lower triangle in every lane
  {
    float ic[10] = {Ib.m, Ib.h[0], Ib.h[1], Ib.h[2], Ib.I[0], Ib.I[1], Ib.I[2], Ib.I[3], Ib.I[4], Ib.I[5]};
    suffix_sum<10>(ic);
    SI In;  // Ic_{k+1}
    In.m = dppzf<DPP_SHL + 1>(ic[0]);
#pragma unroll
    for (int a = 0; a < 3; ++a) In.h[a] = dppzf<DPP_SHL + 1>(ic[1 + a]);
#pragma unroll
    for (int a = 0; a < 6; ++a) In.I[a] = dppzf<DPP_SHL + 1>(ic[4 + a]);
    float Fk[6], Mk[ND];
    si_mul(In, Sown, Fk);
#pragma unroll
    for (int jj = 0; jj < ND; ++jj) {
      float t = 0.f;
#pragma unroll
      for (int a = 0; a < 6; ++a) t += S[jj][a] * Fk[a];
      Mk[jj] = t;
    }
    // this lane's row of M (own_lane): joint row 6 + s from its own column (lanes 0-5), root row
    // s - 6 of the Ic_0 block (lane 0's composite) in lanes 6-11
    {
      const float m0t = tb<0>(ic[0]), hx = tb<0>(ic[1]), hy = tb<0>(ic[2]), hz = tb<0>(ic[3]);
      const float i0 = tb<0>(ic[4]), i1 = tb<0>(ic[5]), i2 = tb<0>(ic[6]);
      const float i3 = tb<0>(ic[7]), i4 = tb<0>(ic[8]), i5 = tb<0>(ic[9]);
      const int r = q.s - 6;
      // lower triangle of root row r (entries past the diagonal unused). One select per statement:
      // written as nested ?: chains, clang emitted branches that SimplifyCFG folded into a
      // compare-and-branch tree on r with out-of-line blocks (~100 scalar instructions per substep)
      float B[6];
      B[0] = hy;
      B[0] = r == 4 ? -hz : B[0];
      B[0] = r == 3 ? 0.f : B[0];
      B[0] = r == 2 ? i4 : B[0];
      B[0] = r == 1 ? i3 : B[0];
      B[0] = r == 0 ? i0 : B[0];
      B[1] = -hx;
      B[1] = r == 4 ? 0.f : B[1];
      B[1] = r == 3 ? hz : B[1];
      B[1] = r == 2 ? i5 : B[1];
      B[1] = r == 1 ? i1 : B[1];
      B[2] = r == 4 ? hx : 0.f;
      B[2] = r == 3 ? -hy : B[2];
      B[2] = r == 2 ? i2 : B[2];
      B[3] = r == 3 ? m0t : 0.f;
      B[4] = r == 4 ? m0t : 0.f;
      B[5] = r == 5 ? m0t : 0.f;
      const bool jrow = q.s < ND;
#pragma unroll
      for (int a = 0; a < 6; ++a) R[a] = jrow ? Fk[a] : B[a];
#pragma unroll
      for (int jj = 0; jj < ND; ++jj) R[6 + jj] = jrow ? Mk[jj] + (jj == q.s ? arm : 0.f) : 0.f;
    }
  }
  }  // S

  // implicit PD drives. Pass 1: all implicit (armature arm = dt kd + dt^2 kp on the joint
  // diagonal; the drive adds arm qd + dt (kp (q* - q) - (kd + dt kp) qd) to the joint rows of the
  // right-hand side). A joint whose implicit torque exceeds the effort limit gets an explicit
  // +-limit torque and loses its armature, then the trailing rows are re-solved.
  sp.mark(3);
  float Li[NV];
  // this lane's M row entries of the joint columns, kept for a re-factorisation of the trailing
  // block if a drive saturates (the contact-row granules are dead until the rows are rebuilt)
  float4* stash = q.b + STASH_OFF + 2 * q.lane;
  stash[0] = make_float4(R[6], R[7], R[8], R[9]);
  stash[1] = make_float4(R[10], R[11], 0.f, 0.f);
  cholesky_team(R, L, Li);
  float rhs[ND], padd[ND];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    rhs[j] = m->kp * (target[j] - s.jq[j]) - (m->kd + dt * m->kp) * s.jqd[j];
    padd[j] = fmaf(arm, s.jqd[j], dt * rhs[j]);
  }
  // whitened free velocity w = L^-1 ((M + A) u + dt (tau - C)) by team forward substitution;
  // lane s keeps coordinate own_row(s) as its Gauss-Seidel coordinate wd
  float t = yown + pick_lane<ND>(padd, q.s);
  float z[NV], wd = 0.f;
  team_fwd<0, 6>(R, Li, t, z, wd, q.s);
  const float t5 = t;  // joint rows after the root columns (a saturated drive restarts here)
  team_fwd<6, NV>(R, Li, t, z, wd, q.s);
  {
    // joint part of the free velocity (L^-T w restricted to the trailing block) for the
    // saturation test
    float uf[NV];
#pragma unroll
    for (int i = NV - 1; i >= 6; --i) {
      float tt = z[i];
#pragma unroll
      for (int k = i + 1; k < NV; ++k) tt -= L[tri(k, i)] * uf[k];
      uf[i] = tt * Li[i];
    }
    unsigned sat = 0;
    float dsat[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float tau = rhs[j] - (arm / dt) * (uf[6 + j] - s.jqd[j]);
      const bool sj = tau > m->effort_limit || tau < -m->effort_limit;
      sat |= sj ? 1u << j : 0u;
      // joint row j without the drive: - arm qd - dt rhs, with the explicit +-limit torque
      dsat[j] = sj ? dt * ((tau > 0.f ? m->effort_limit : -m->effort_limit) - rhs[j]) - arm * s.jqd[j] : 0.f;
    }
    if (sat) {
      // M changes only on the saturated joints' diagonals (joint coordinates 6..11, the last
      // ones), so L's leading columns and z[0..5] are unchanged: re-factor the trailing 6x6 block
      // from the stashed rows (= the oracle's full re-factorisation) and redo the trailing steps
      // of the forward substitution from the joint rows' state after the root columns
      const float4 s0 = stash[0], s1 = stash[1];
      const float rt[ND] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y};
#pragma unroll
      for (int jj = 0; jj < ND; ++jj) R[6 + jj] = rt[jj] - ((((sat >> jj) & 1u) != 0u && q.s == jj) ? arm : 0.f);
      team_chol_col<6>(R, L, Li); team_chol_col<7>(R, L, Li); team_chol_col<8>(R, L, Li);
      team_chol_col<9>(R, L, Li); team_chol_col<10>(R, L, Li); team_chol_col<11>(R, L, Li);
      t = t5 + pick_lane<ND>(dsat, q.s);
      team_fwd<6, NV>(R, Li, t, z, wd, q.s);
    }
  }

  sp.mark(4);
  // contact rows (lane s builds slot s): Y = L^-1 J^T (whitened), effective masses, the
  // normal/tangent cross terms and the bias velocity. J of direction d at point x on body b:
  // [x x d ; d ; d.(a_j x (x - o_j)) for joints j < b]
  // The candidates share storage with the rows (region U): every lane reads its candidate, then
  // the wave writes. The normal + code go to FRC for the contact sensor.
  // TGS-style solve (cfg.solver_mode 1): solver_iterations sub-iterations of h = dt / iterations,
  // each one sweep whose biases come from the contact's separation advanced by h times its normal
  // velocity after the previous sub-iteration; lane c keeps slot c's separation in sep_own
  constexpr bool tgs = kTgs;
  const float hsub = dt / (float)cfg.solver_iterations;
  float sep_own = 0.f;
  int rim_own = -1, gl_own = 0;  // kRefresh: slot q.s's ground link and rim candidate (4 ci + r)
  float anc[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // kRefresh, solver_mode 3: slot q.s's self-contact anchors
  if (q.s < nc) {
    const int c = q.s;
    const int pos = over ? q.map(c) : c;
    float S[ND][6], org[ND][3];
    read_joints(q, S, org);
    const float4 g0 = q.cand(pos, 0), gn = q.cand(pos, 1);
    wave_sync();  // (all active lanes execute this together: the wave's reads precede its writes)
    q.frc(c) = gn;
    q.yg_zero(c) = make_float4(0.f, 0.f, 0.f, 0.f);
    const float x[3] = {g0.x, g0.y, g0.z};
    const float n[3] = {gn.x, gn.y, gn.z};
    const float sep = g0.w;
    const int code = (int)gn.w;
    const int ba = link_body(code >> 4);
    const int lb = (code & 15) - 1;
    const int bb = lb >= 0 ? link_body(lb) : -1;
    if (kRefresh && lb < 0) {
      // which rim candidate detect made this point from: the nearest of the link's 8 at this pose
      gl_own = code >> 4;
      float best = 3.4e38f;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float xc[3];
        ground_rim_point(q, gl_own, k >> 2, k & 3, xc);
        const float d2 = (xc[0] - x[0]) * (xc[0] - x[0]) + (xc[1] - x[1]) * (xc[1] - x[1]) + (xc[2] - x[2]) * (xc[2] - x[2]);
        if (d2 < best) { best = d2; rim_own = k; }
      }
    }
    if (kRefresh && lb >= 0 && cfg.solver_mode == 3) {
      // the self contact's body-fixed anchors x +- n sep / 2 on A / B (oracle substep, `anc`)
#pragma unroll
      for (int e = 0; e < 2; ++e) {
        float R[9], p[3];
        read_frame(q, e ? bb : ba, R, p);
        const float hs = e ? -0.5f * sep : 0.5f * sep;
        const float d[3] = {x[0] + hs * n[0] - p[0], x[1] + hs * n[1] - p[1], x[2] + hs * n[2] - p[2]};
#pragma unroll
        for (int a = 0; a < 3; ++a) anc[3 * e + a] = R[a] * d[0] + R[3 + a] * d[1] + R[6 + a] * d[2];
      }
    }
    // per-joint lever vectors a_j x (x - o_j), signed by which side of the contact the joint is on
    float cj[ND][3];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float xo[3] = {x[0] - org[j][0], x[1] - org[j][1], x[2] - org[j][2]};
      float c3[3];
      cross3(S[j], xo, c3);
      const float sg = (j < ba ? 1.f : 0.f) - (j < bb ? 1.f : 0.f);
      cj[j][0] = sg * c3[0]; cj[j][1] = sg * c3[1]; cj[j][2] = sg * c3[2];
    }
    const float root = bb >= 0 ? 0.f : 1.f;  // self contacts: the root terms cancel
    float t1[3], t2[3];
    tangents(n, t1, t2);
    float invm[3], Y[3][NV];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      float d[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) d[a] = r == 0 ? n[a] : (r == 1 ? t1[a] : t2[a]);
      float J[NV];
      float xd[3];
      cross3(x, d, xd);
      J[0] = root * xd[0]; J[1] = root * xd[1]; J[2] = root * xd[2];
      J[3] = root * d[0]; J[4] = root * d[1]; J[5] = root * d[2];
#pragma unroll
      for (int j = 0; j < ND; ++j) J[6 + j] = dot3(cj[j], d);
      fwd_sub(L, Li, J, Y[r]);
      invm[r] = 1.f / (dot12(Y[r], Y[r]) + 1e-9f);
    }
#pragma unroll
    for (int d = 0; d < NV; ++d) q.yg_at(c, own_lane(d)) = make_float4(Y[0][d], Y[1][d], Y[2][d], 0.f);
    sep_own = sep;
    const float vmin = contact_bias(cfg, m, sep, tgs ? hsub : dt, dt);
    q.aux(c, 0) = make_float4(invm[0], invm[1], invm[2], vmin * invm[0]);
    // friction combine mode "multiply": ground (terrain coefficient) x link, link x link
    // (the static coefficient is raised to the dynamic one where the independent DR draws put it
    // below, as PhysX's material combine does)
    const float mu_cd = kLinkFriction ? q.fricd(code >> 4) * (lb >= 0 ? q.fricd(lb) : cfg.friction_dynamic) : 0.f;
    const float mu_c = kLinkFriction ? fmaxf(q.fric(code >> 4) * (lb >= 0 ? q.fric(lb) : cfg.friction), mu_cd) : 0.f;
    q.aux(c, 1) = make_float4(dot12(Y[1], Y[0]) * invm[1], dot12(Y[2], Y[0]) * invm[2], mu_c, mu_cd);
    q.lam(c) = make_float4(0.f, 0.f, 0.f, 0.f);
  }
  wave_sync();
  if (q.s >= nc && q.s < NCM) {
    // an unused slot is an exact no-op update (zero rows, effective masses and bias: the impulse
    // stays 0 and w is unchanged), so the sweep needs no per-env mask. (Region U: written only
    // after every active lane has read its candidate above.)
    const int c = q.s;
#pragma unroll
    for (int d = 0; d < NV; ++d) q.yg_at(c, d) = make_float4(0.f, 0.f, 0.f, 0.f);
    q.yg_zero(c) = make_float4(0.f, 0.f, 0.f, 0.f);
    q.aux(c, 0) = make_float4(0.f, 0.f, 0.f, 0.f);
    q.aux(c, 1) = make_float4(0.f, 0.f, 0.f, 0.f);
    q.lam(c) = make_float4(0.f, 0.f, 0.f, 0.f);
    q.frc(c) = make_float4(0.f, 0.f, 0.f, -1.f);  // no contact: the next substep's GJK starts cold
  }
  wave_sync();

  sp.mark(5);
  // projected Gauss-Seidel on the whitened velocity (Coulomb disk friction); lane s owns
  // coordinate own_row(s) of w (its granule of every contact row holds that coordinate).
  float w[NV];
  float wsum_own;  // TGS: this lane's coordinate of the sub-iterations' mean w
  // Sweeps outer, the NCM slots unrolled inner: constant LDS offsets, slot c + 1's granules read
  // while slot c updates, slots c >= the wave's largest contact count skipped uniformly, the
  // slots between an env's own count and that maximum are no-op updates (zeroed above). The
  // impulses are team-uniform (every lane computes the same update, and every lane stores it).
  {
    const float mu_d = cfg.friction_dynamic, mu = fmaxf(cfg.friction, mu_d);
    const float4* yl = q.b + YG_OFF + q.ygl();
    const int ncw = max(max(__builtin_amdgcn_readlane(nc, 0), __builtin_amdgcn_readlane(nc, TL)),
                        max(__builtin_amdgcn_readlane(nc, 2 * TL), __builtin_amdgcn_readlane(nc, 3 * TL)));
    float wsum = 0.f;  // TGS: the sum of the sub-iterations' w (this lane's coordinate)
    for (int it = 0; it < cfg.solver_iterations; ++it) {
      if (tgs && it > 0) {  // re-linearise the biases
        // every contact's normal velocity Y0_c . w at once (round 6): w broadcast to the team, lane c
        // reads its slot's 12 granules -- one short chain instead of a team reduction per contact
        const float wb[NV] = {tb<own_lane(0)>(wd), tb<own_lane(1)>(wd), tb<own_lane(2)>(wd), tb<own_lane(3)>(wd),
                              tb<own_lane(4)>(wd), tb<own_lane(5)>(wd), tb<own_lane(6)>(wd), tb<own_lane(7)>(wd),
                              tb<own_lane(8)>(wd), tb<own_lane(9)>(wd), tb<own_lane(10)>(wd), tb<own_lane(11)>(wd)};
        if (q.s < nc) {
          float vn = 0.f;
#pragma unroll
          for (int d = 0; d < NV; ++d) vn = fmaf(q.yg_at(q.s, own_lane(d)).x, wb[d], vn);
          sep_own = fmaf(hsub, vn, sep_own);
          const float4 a0 = q.aux(q.s, 0);
          q.aux(q.s, 0) = make_float4(a0.x, a0.y, a0.z, contact_bias(cfg, m, sep_own, hsub, dt) * a0.x);
        }
        wave_sync();
        if (kRefresh) refresh_contacts(cfg, m, s, q, L, Li, wsum / (float)it, (float)it * hsub, hsub, dt, nc, rim_own,
                                       gl_own, anc, sep_own);
      }
      float4 G = q.yg(yl, 0), X = q.aux(0, 0), Z = q.aux(0, 1), La = q.lam(0);
#pragma unroll
      for (int c = 0; c < NCM; ++c) {
        const int cn = c + 1 < NCM ? c + 1 : c;
        const float4 Gn = q.yg(yl, cn), Xn = q.aux(cn, 0), Zn = q.aux(cn, 1), Ln = q.lam(cn);
        if (c < ncw) {
          const float4 nA = pgs_update(G, X, Z, La, kLinkFriction ? Z.z : mu, kLinkFriction ? Z.w : mu_d, wd);
          // every lane of the team stores the same impulse to the same address (team-uniform:
          // identical bits in all 16 lanes; an LDS write to one address is not a bank conflict), so
          // the store needs no exec-mask switch around it
          q.lam(c) = nA;
        }
        G = Gn; X = Xn; Z = Zn; La = Ln;
      }
      wsum += wd;
    }
    w[0] = tb<own_lane(0)>(wd); w[1] = tb<own_lane(1)>(wd); w[2] = tb<own_lane(2)>(wd);
    w[3] = tb<own_lane(3)>(wd); w[4] = tb<own_lane(4)>(wd); w[5] = tb<own_lane(5)>(wd);
    w[6] = tb<own_lane(6)>(wd); w[7] = tb<own_lane(7)>(wd); w[8] = tb<own_lane(8)>(wd);
    w[9] = tb<own_lane(9)>(wd); w[10] = tb<own_lane(10)>(wd); w[11] = tb<own_lane(11)>(wd);
    wsum_own = wsum * (1.f / (float)cfg.solver_iterations);
  }
  wave_sync();  // last impulses visible to every lane
  sp.mark(6);
  float un[NV];
  bwd_sub(L, Li, w, un);

  if (last) {
    // ContactSensor inputs: net force on the feet, max |net force| over undesired links.
    // Lane s forms the force of slot s (into AUX, dead after the PGS: FRC keeps the normals for the
    // next substep's GJK warm start), then sums the env's contacts onto link s.
    if (q.s < nc) {
      const float4 gn = q.frc(q.s), lam = q.lam(q.s);
      const float n[3] = {gn.x, gn.y, gn.z};
      float t1[3], t2[3];
      tangents(n, t1, t2);
      float f[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) f[a] = (lam.x * n[a] + lam.y * t1[a] + lam.z * t2[a]) / dt;
      q.aux(q.s, 0) = make_float4(f[0], f[1], f[2], gn.w);
    }
    wave_sync();
    float Fl[3] = {0.f, 0.f, 0.f};
    for (int c = 0; c < nc; ++c) {
      const float4 f = q.aux(c, 0);
      const int code = (int)f.w;
      const int la = code >> 4, lb = (code & 15) - 1;
      const float sa = (q.s == la ? 1.f : 0.f) - (q.s == lb ? 1.f : 0.f);
      Fl[0] += sa * f.x; Fl[1] += sa * f.y; Fl[2] += sa * f.z;
    }
    const float fm = (q.s >= 1 && q.s <= 10) ? sqrtf(dot3(Fl, Fl)) : 0.f;
    so.undes_fmax = tmax(fm);
#pragma unroll
    for (int a = 0; a < 3; ++a) { so.feet_f[0][a] = tb<0>(Fl[a]); so.feet_f[1][a] = tb<11>(Fl[a]); }
    if (kDebugForces) { dbgF[0][0] = Fl[0]; dbgF[0][1] = Fl[1]; dbgF[0][2] = Fl[2]; }
  }

  clamp_speeds(m, un);
  // semi-implicit Euler (root twist at P -> classical root-origin velocity adds omega x v dt): the
  // new velocity, then the pose integrated with the pose velocity (PGS: the new velocity; TGS:
  // the mean of the sub-iterations' velocities, u = L^-T of the mean w)
  float wv[3];
  cross3(s.av, s.lv, wv);
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    s.av[a] = un[a];
    s.lv[a] = un[3 + a] + dt * wv[a];
  }
#pragma unroll
  for (int j = 0; j < ND; ++j) s.jqd[j] = un[6 + j];
  if (tgs) {
    w[0] = tb<own_lane(0)>(wsum_own); w[1] = tb<own_lane(1)>(wsum_own); w[2] = tb<own_lane(2)>(wsum_own);
    w[3] = tb<own_lane(3)>(wsum_own); w[4] = tb<own_lane(4)>(wsum_own); w[5] = tb<own_lane(5)>(wsum_own);
    w[6] = tb<own_lane(6)>(wsum_own); w[7] = tb<own_lane(7)>(wsum_own); w[8] = tb<own_lane(8)>(wsum_own);
    w[9] = tb<own_lane(9)>(wsum_own); w[10] = tb<own_lane(10)>(wsum_own); w[11] = tb<own_lane(11)>(wsum_own);
    bwd_sub(L, Li, w, un);
    clamp_speeds(m, un);
  }
#pragma unroll
  for (int a = 0; a < 3; ++a) s.pos[a] += dt * (un[3 + a] + dt * wv[a]);
  {
    const float th = sqrtf(un[0] * un[0] + un[1] * un[1] + un[2] * un[2]) * dt;
    float dq[4];
    if (th > 1e-12f) {
      float sn, cs;
      sincos_r(0.5f * th, &sn, &cs);
      const float sc = sn / th * dt;
      dq[0] = cs; dq[1] = un[0] * sc; dq[2] = un[1] * sc; dq[3] = un[2] * sc;
    } else {
      dq[0] = 1.f; dq[1] = 0.5f * dt * un[0]; dq[2] = 0.5f * dt * un[1]; dq[3] = 0.5f * dt * un[2];
    }
    float qn[4];
    qmul(dq, s.quat, qn);
    qnormalize(qn);
    s.quat[0] = qn[0]; s.quat[1] = qn[1]; s.quat[2] = qn[2]; s.quat[3] = qn[3];
  }
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const float qv = s.jq[j] + dt * un[6 + j];
    // (the wrap as selects: written as if / else if it compiled to two divergent branches per joint)
    const float qd = qv - 2.f * TWO_PI_F, qu = qv + 2.f * TWO_PI_F;
    float qw = qv < -TWO_PI_F ? qu : qv;
    qw = qv > TWO_PI_F ? qd : qw;
    s.jq[j] = qw;
  }
}

// ------------------------------------------------------------------------- MDP helpers
struct Cache {
  float base_pos[3], base_quat[4], fwd[3], heading_err, vfwd;
  float feet_pos[2][3], feet_z[2][3], feet_x[2][3];
};

__device__ __forceinline__ void link_pose(MP m, const Kin& k, int l, float pos[3],
                                          float quat[4]) {
  const int b = link_body(l);
  float t[3];
  float lp[3], lr[4];
  ldc(lp, m->link_pos[l]);
  ldc(lr, m->link_rot[l]);
  mv3(k.R[b], lp, t);
  pos[0] = k.p[b][0] + t[0]; pos[1] = k.p[b][1] + t[1]; pos[2] = k.p[b][2] + t[2];
  qmul(k.q[b], lr, quat);
}

__device__ __forceinline__ void link_com_vel(MP m, const Kin& k, const float V[NB][6], int l,
                                             float v[3]) {
  const int b = link_body(l);
  float c[3];
  float lc[3];
  ldc(lc, m->link_com[l]);
  mv3(k.R[b], lc, c);
  c[0] += k.p[b][0]; c[1] += k.p[b][1]; c[2] += k.p[b][2];
  float wc[3];
  cross3(V[b], c, wc);
  v[0] = V[b][3] + wc[0]; v[1] = V[b][4] + wc[1]; v[2] = V[b][5] + wc[2];
}

// the _get_observations cache (v2.py:315-345) of a physics state
__device__ __forceinline__ void make_cache(MP m, const Phys& s, Cache& o) {
  Kin k;
  fk(m, s, k);
  float V[NB][6];
  body_vel(k, s, V);
  constexpr int BASE = 6, F0 = 0, F1 = 11;
  float bq[4], fq[2][4], bv[3];
  link_pose(m, k, BASE, o.base_pos, bq);
  link_pose(m, k, F0, o.feet_pos[0], fq[0]);
  link_pose(m, k, F1, o.feet_pos[1], fq[1]);
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    o.base_pos[a] += s.pos[a];
    o.feet_pos[0][a] += s.pos[a];
    o.feet_pos[1][a] += s.pos[a];
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) o.base_quat[a] = bq[a];
  link_com_vel(m, k, V, BASE, bv);
  float R[9];
  qmat(bq, R);
  const float sh[3] = {R[2], R[5], R[8]};              // quat_apply(base_quat, z)  v2.py:322
  o.fwd[0] = sh[1];                                     // (0,0,-1) x sh              v2.py:323
  o.fwd[1] = -sh[0];
  o.fwd[2] = 0.f * sh[0];
  o.heading_err = -o.fwd[1];                            // v2.py:324
  o.vfwd = dot3(bv, o.fwd);                             // v2.py:326-327
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    qmat(fq[f], R);
    const float sg = f == 0 ? 1.f : -1.f;               // axis_z_feet = (0,0,1),(0,0,-1) v2.py:341-343
    o.feet_z[f][0] = sg * R[2]; o.feet_z[f][1] = sg * R[5]; o.feet_z[f][2] = sg * R[8];
    o.feet_x[f][0] = R[0]; o.feet_x[f][1] = R[3]; o.feet_x[f][2] = R[6];  // axis_x_feet v2.py:338-340
  }
}

// link l's world pose (position relative to P, quaternion) from the published body pose
__device__ __forceinline__ void link_pose_q(MP m, const Q& q, int l, float pos[3], float quat[4]) {
  const int b = link_body(l);
  float R[9], p[3];
  read_frame(q, b, R, p);
  const float4 bq = q.body(b, 3);
  const float qb[4] = {bq.x, bq.y, bq.z, bq.w};
  float t[3], lp[3], lr[4];
  ldc(lp, m->link_pos[l]);
  ldc(lr, m->link_rot[l]);
  mv3(R, lp, t);
  pos[0] = p[0] + t[0]; pos[1] = p[1] + t[1]; pos[2] = p[2] + t[2];
  qmul(qb, lr, quat);
}

// world linear velocity of the point lc (body frame of body b): body b's twist at P from the
// joint rates, then v + w x c
__device__ __forceinline__ void body_point_vel_q(const Q& q, const Phys& s, const float S[ND][6], int b,
                                                 const float lc[3], float v[3]) {
  float V[6] = {s.av[0], s.av[1], s.av[2], s.lv[0], s.lv[1], s.lv[2]};
#pragma unroll
  for (int j = 0; j < ND; ++j)
    if (j < b)
#pragma unroll
      for (int a = 0; a < 6; ++a) V[a] += S[j][a] * s.jqd[j];
  float R[9], p[3], c[3];
  read_frame(q, b, R, p);
  mv3(R, lc, c);
  c[0] += p[0]; c[1] += p[1]; c[2] += p[2];
  float wc[3];
  cross3(V, c, wc);
  v[0] = V[3] + wc[0]; v[1] = V[4] + wc[1]; v[2] = V[5] + wc[2];
}

// world linear velocity of link l's frame origin (body_link_lin_vel_w, standup.py:774-856)
__device__ __forceinline__ void link_origin_vel_q(MP m, const Q& q, const Phys& s, const float S[ND][6], int l,
                                                  float v[3]) {
  float lp[3];
  ldc(lp, m->link_pos[l]);
  body_point_vel_q(q, s, S, link_body(l), lp, v);
}

// world linear velocity of link l's COM: body b's twist at P from the joint rates, then v + w x c
__device__ __forceinline__ void link_com_vel_q(MP m, const Q& q, const Phys& s, const float S[ND][6], int l,
                                               float v[3]) {
  const int b = link_body(l);
  float V[6] = {s.av[0], s.av[1], s.av[2], s.lv[0], s.lv[1], s.lv[2]};
#pragma unroll
  for (int j = 0; j < ND; ++j)
    if (j < b)
#pragma unroll
      for (int a = 0; a < 6; ++a) V[a] += S[j][a] * s.jqd[j];
  float R[9], p[3], lc[3], c[3];
  read_frame(q, b, R, p);
  ldc(lc, m->link_com[l]);
  mv3(R, lc, c);
  c[0] += p[0]; c[1] += p[1]; c[2] += p[2];
  float wc[3];
  cross3(V, c, wc);
  v[0] = V[3] + wc[0]; v[1] = V[4] + wc[1]; v[2] = V[5] + wc[2];
}

// the _get_observations cache (v2.py:315-345) of a physics state, from the published poses
// (call after fk_team + a barrier)
__device__ __forceinline__ void make_cache_q(MP m, const Q& q, const Phys& s, Cache& o) {
  constexpr int BASE = 6, F0 = 0, F1 = 11;
  float S[ND][6], org[ND][3];
  read_joints(q, S, org);
  float bq[4], fq[2][4], bv[3];
  link_pose_q(m, q, BASE, o.base_pos, bq);
  link_pose_q(m, q, F0, o.feet_pos[0], fq[0]);
  link_pose_q(m, q, F1, o.feet_pos[1], fq[1]);
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    o.base_pos[a] += s.pos[a];
    o.feet_pos[0][a] += s.pos[a];
    o.feet_pos[1][a] += s.pos[a];
  }
#pragma unroll
  for (int a = 0; a < 4; ++a) o.base_quat[a] = bq[a];
  link_com_vel_q(m, q, s, S, BASE, bv);
  float R[9];
  qmat(bq, R);
  const float sh[3] = {R[2], R[5], R[8]};              // quat_apply(base_quat, z)  v2.py:322
  o.fwd[0] = sh[1];                                     // (0,0,-1) x sh              v2.py:323
  o.fwd[1] = -sh[0];
  o.fwd[2] = 0.f * sh[0];
  o.heading_err = -o.fwd[1];                            // v2.py:324
  o.vfwd = dot3(bv, o.fwd);                             // v2.py:326-327
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    qmat(fq[f], R);
    const float sg = f == 0 ? 1.f : -1.f;               // axis_z_feet = (0,0,1),(0,0,-1) v2.py:341-343
    o.feet_z[f][0] = sg * R[2]; o.feet_z[f][1] = sg * R[5]; o.feet_z[f][2] = sg * R[8];
    o.feet_x[f][0] = R[0]; o.feet_x[f][1] = R[3]; o.feet_x[f][2] = R[6];  // axis_x_feet v2.py:338-340
  }
}

struct Mdp {
  float p_delta[ND], actions[ND];
  float down_pos[2][3], step_len[2], f_last[2];
  float heading_sum, yerr_sum, force_sum;
  float fz_hist[ZB_HIST][2], fmax_hist[ZB_HIST];
  float air_cur[2], air_last[2], contact_cur[2];
  float ep_len;
  float sums[ZB_NUM_REWARD_TERMS];
};

__device__ __forceinline__ void load_state(const float* __restrict__ st, int N, int i, Phys& p, Mdp& d) {
#define LD(f) st[(size_t)(f) * N + i]
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.pos[a] = LD(ZB_S_ROOT_POS + a); p.lv[a] = LD(ZB_S_ROOT_LINVEL + a); p.av[a] = LD(ZB_S_ROOT_ANGVEL + a); }
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = LD(ZB_S_ROOT_QUAT + a);
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    p.jq[j] = LD(ZB_S_JOINT_POS + j); p.jqd[j] = LD(ZB_S_JOINT_VEL + j);
    d.p_delta[j] = LD(ZB_S_P_DELTA + j); d.actions[j] = LD(ZB_S_ACTIONS + j);
  }
#pragma unroll
  for (int f = 0; f < 2; ++f) {
#pragma unroll
    for (int a = 0; a < 3; ++a) d.down_pos[f][a] = LD(ZB_S_FEET_DOWN_POS + 3 * f + a);
    d.step_len[f] = LD(ZB_S_FEET_STEP_LEN + f);
    d.f_last[f] = LD(ZB_S_FEET_F_LAST + f);
    d.air_cur[f] = LD(ZB_S_FEET_AIR_CUR + f);
    d.air_last[f] = LD(ZB_S_FEET_AIR_LAST + f);
    d.contact_cur[f] = LD(ZB_S_FEET_CONTACT_CUR + f);
  }
  d.heading_sum = LD(ZB_S_HEADING_SUM);
  d.yerr_sum = LD(ZB_S_Y_ERR_SUM);
  d.force_sum = LD(ZB_S_FEET_FORCE_SUM);
#pragma unroll
  for (int h = 0; h < ZB_HIST; ++h) {
    d.fz_hist[h][0] = LD(ZB_S_FEET_FZ_HIST + 2 * h);
    d.fz_hist[h][1] = LD(ZB_S_FEET_FZ_HIST + 2 * h + 1);
    d.fmax_hist[h] = LD(ZB_S_UNDES_FMAX_HIST + h);
  }
  d.ep_len = LD(ZB_S_EP_LEN);
#pragma unroll
  for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) d.sums[t] = LD(ZB_S_EP_SUMS + t);
#undef LD
}

__device__ __forceinline__ void store_state(float* __restrict__ st, int N, int i, const Phys& p, const Mdp& d) {
#define SV(f, v) st[(size_t)(f) * N + i] = (v)
#pragma unroll
  for (int a = 0; a < 3; ++a) { SV(ZB_S_ROOT_POS + a, p.pos[a]); SV(ZB_S_ROOT_LINVEL + a, p.lv[a]); SV(ZB_S_ROOT_ANGVEL + a, p.av[a]); }
#pragma unroll
  for (int a = 0; a < 4; ++a) SV(ZB_S_ROOT_QUAT + a, p.quat[a]);
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    SV(ZB_S_JOINT_POS + j, p.jq[j]); SV(ZB_S_JOINT_VEL + j, p.jqd[j]);
    SV(ZB_S_P_DELTA + j, d.p_delta[j]); SV(ZB_S_ACTIONS + j, d.actions[j]);
  }
#pragma unroll
  for (int f = 0; f < 2; ++f) {
#pragma unroll
    for (int a = 0; a < 3; ++a) SV(ZB_S_FEET_DOWN_POS + 3 * f + a, d.down_pos[f][a]);
    SV(ZB_S_FEET_STEP_LEN + f, d.step_len[f]);
    SV(ZB_S_FEET_F_LAST + f, d.f_last[f]);
    SV(ZB_S_FEET_AIR_CUR + f, d.air_cur[f]);
    SV(ZB_S_FEET_AIR_LAST + f, d.air_last[f]);
    SV(ZB_S_FEET_CONTACT_CUR + f, d.contact_cur[f]);
  }
  SV(ZB_S_HEADING_SUM, d.heading_sum);
  SV(ZB_S_Y_ERR_SUM, d.yerr_sum);
  SV(ZB_S_FEET_FORCE_SUM, d.force_sum);
#pragma unroll
  for (int h = 0; h < ZB_HIST; ++h) {
    SV(ZB_S_FEET_FZ_HIST + 2 * h, d.fz_hist[h][0]);
    SV(ZB_S_FEET_FZ_HIST + 2 * h + 1, d.fz_hist[h][1]);
    SV(ZB_S_UNDES_FMAX_HIST + h, d.fmax_hist[h]);
  }
  SV(ZB_S_EP_LEN, d.ep_len);
#pragma unroll
  for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) SV(ZB_S_EP_SUMS + t, d.sums[t]);
#undef SV
}

__device__ __forceinline__ void phys_default(MP m, Phys& p) {
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.pos[a] = m->default_root_pos[a]; p.lv[a] = 0.f; p.av[a] = 0.f; }
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = m->default_root_quat[a];
#pragma unroll
  for (int j = 0; j < ND; ++j) { p.jq[j] = m->default_joint_pos[j]; p.jqd[j] = 0.f; }
}

// feet link origins (env-local world) of a physical state (one lane per env)
__device__ __forceinline__ void feet_world(MP m, const Phys& p, float out[2][3]) {
  Kin k;
  fk(m, p, k);
  float fq[4];
  link_pose(m, k, m->foot_links[0], out[0], fq);
  link_pose(m, k, m->foot_links[1], out[1], fq);
#pragma unroll
  for (int a = 0; a < 3; ++a) { out[0][a] += p.pos[a]; out[1][a] += p.pos[a]; }
}

// _reset_idx for one env (v2.py:413-459); feet_step_len and f_last are NOT reset (reference).
// feet_down_pos_last = the pre-reset feet positions (v2.py:436), or with `refresh`
// the feet positions of the default pose (dflt[0], dflt[1], zb_derive_kernel).
__device__ __forceinline__ void reset_env(MP m, const float4* dflt, Phys& p, Mdp& d, int refresh) {
  float pre[2][3];
  if (!refresh) feet_world(m, p, pre);
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.pos[a] = m->default_root_pos[a]; p.lv[a] = 0.f; p.av[a] = 0.f; }
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = m->default_root_quat[a];
#pragma unroll
  for (int j = 0; j < ND; ++j) { p.jq[j] = m->default_joint_pos[j]; p.jqd[j] = 0.f; d.p_delta[j] = 0.f; d.actions[j] = 0.f; }
  if (refresh) {
    const float4 f0 = dflt[0], f1 = dflt[1];
    d.down_pos[0][0] = f0.x; d.down_pos[0][1] = f0.y; d.down_pos[0][2] = f0.z;
    d.down_pos[1][0] = f1.x; d.down_pos[1][1] = f1.y; d.down_pos[1][2] = f1.z;
  } else {
#pragma unroll
    for (int f = 0; f < 2; ++f)
#pragma unroll
      for (int a = 0; a < 3; ++a) d.down_pos[f][a] = pre[f][a];
  }
  d.heading_sum = 0.f;
  d.yerr_sum = 0.f;
  d.force_sum = 0.f;  // v2.py:437
#pragma unroll
  for (int h = 0; h < ZB_HIST; ++h) { d.fz_hist[h][0] = d.fz_hist[h][1] = 0.f; d.fmax_hist[h] = 0.f; }
#pragma unroll
  for (int f = 0; f < 2; ++f) { d.air_cur[f] = d.air_last[f] = d.contact_cur[f] = 0.f; }
  d.ep_len = 0.f;
#pragma unroll
  for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) d.sums[t] = 0.f;
}

__device__ __forceinline__ void write_obs(MP m, const Phys& p, const Mdp& d,
                                          float* __restrict__ obs, int i) {
  Cache c;
  make_cache(m, p, c);
  float* o = obs + (size_t)i * ZB_OBS_DIM;
  o[0] = c.base_quat[0]; o[1] = c.base_quat[1]; o[2] = c.base_quat[2]; o[3] = c.base_quat[3];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    o[4 + j] = p.jq[j] - m->default_joint_pos[j];
    o[10 + j] = p.jqd[j];
    o[16 + j] = d.actions[j];
  }
  o[22] = 1.0f;
}

// accumulator layout: [0..15] episode-sum totals of reset envs, then n_reset, n_died, n_timeout
// (the manager env also counts a second termination term and averages its two command metrics)
constexpr int ACC_NRES = ZB_MAX_REWARD_TERMS, ACC_DIED = ACC_NRES + 1, ACC_TOUT = ACC_NRES + 2;
constexpr int ACC_TERM2 = ACC_NRES + 3, ACC_MET0 = ACC_NRES + 4, ACC_MET1 = ACC_NRES + 5;
constexpr int ACC = ACC_NRES + 8;
static_assert(ACC == LOGR_W && ACC % 4 == 0, "log row width");
// The episode-log accumulator is ACC_SLOTS copies of the ACC floats, one 128-B line each: a step
// kernel adds into the slot of its workgroup, so the adds of one step spread over many L2 lines
// instead of serialising on one (at a 30 % reset rate one shared line took ~100 us per step);
// zb_finalize_kernel folds the slots and clears them.
constexpr int ACC_STRIDE = 32, ACC_SLOTS = 64;
static_assert(ACC <= ACC_STRIDE, "slot width");
__device__ __forceinline__ float* acc_slot(float* acc, unsigned k) { return acc + (k % ACC_SLOTS) * ACC_STRIDE; }

// Log row of a resetting env: the team lead clears its LDS row and fills the entries it logs.
__device__ __forceinline__ float* log_row(const Q& q) {
  float4* r = reinterpret_cast<float4*>(q.logr(q.e));
#pragma unroll
  for (int k = 0; k < ACC / 4; ++k) r[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  return q.logr(q.e);
}
// Wave-level log reduction (uniform control flow): lane t < ACC adds entry t of the rows of the
// resetting envs of this wave (mask = ballot of their team leads) and issues one atomic into the
// workgroup's slot: at most ACC atomics per wave instead of ACC per resetting env.
__device__ __forceinline__ void log_flush(const Q& q, uint64_t mask, float* acc) {
  if (!mask) return;
  wave_sync();
  if (q.lane < ACC) {
    float v = 0.f;
#pragma unroll
    for (int e = 0; e < EPW; ++e)
      if ((mask >> (e * TL)) & 1ull) v += q.logr(e)[q.lane];
    if (v != 0.f) atomicAdd(acc_slot(acc, blockIdx.x) + q.lane, v);
  }
}

// ------------------------------------------------------------------------- kernels
// Step-end finalisation arguments (zb_finalize_kernel).
constexpr int FIN_FG = 8;  // finalize fold: accumulator slot groups
struct FinArgs {
  float* log_means;
  int32_t* log_counts;
  float* user_means;
  int32_t* user_counts;
  float episode_s;
  uint64_t seed;
  Counters* cnt;
  int ep_len_row;
  float* user_acc;  // zb_set_log_accumulator: += this step's log values (float[ZB_LOG_LEN + ZB_LOG_COUNTS])
};

__device__ __forceinline__ void load_phys(const float* __restrict__ st, int N, int i, Phys& p) {
#define LD(f) st[(size_t)(f) * N + i]
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.pos[a] = LD(ZB_S_ROOT_POS + a); p.lv[a] = LD(ZB_S_ROOT_LINVEL + a); p.av[a] = LD(ZB_S_ROOT_ANGVEL + a); }
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = LD(ZB_S_ROOT_QUAT + a);
#pragma unroll
  for (int j = 0; j < ND; ++j) { p.jq[j] = LD(ZB_S_JOINT_POS + j); p.jqd[j] = LD(ZB_S_JOINT_VEL + j); }
#undef LD
}

// One policy step per lane. Live state across the 4 substeps is kept to the physics state, the
// joint targets and the ~15 floats of the lagged observation cache the rewards need; the MDP
// state is loaded from HBM only after the physics.
template <bool kTgs, bool kRefresh = false, bool kRf = false>
__device__ __forceinline__ void step_body(const zb_model* __restrict__ mg, const float4* __restrict__ links,
                                          zb_task_cfg cfg, int N, float* __restrict__ st,
                                          const float* __restrict__ act, float* __restrict__ obs,
                                          float* __restrict__ rew, uint8_t* __restrict__ term,
                                          uint8_t* __restrict__ trunc, int64_t* __restrict__ done,
                                          float* __restrict__ acc, float* __restrict__ wc, float4* lds) {
  MP m = to_mp(mg);
  const int lane = (int)threadIdx.x;
  const int env = xcd_block(blockIdx.x, gridDim.x) * EPW + lane / TL;
  // a team past N recomputes env N-1 (identical values, identical stores); it never logs
  const int i = env < N ? env : N - 1;
  const bool lead = env < N && lane % TL == 0;
  const Q q = make_q(lds, lane, links);
  for (int t = LNK_G + lane; t < LNK4; t += WGT) lds[LNK_OFF + t] = links[t];
  // the env's state row: lane s loads fields s, s+16, ... (one coalesced load per field group)
  Stamps sp;
  sp.begin();
#define ST(f) st[(size_t)(f) * N + i]
  Phys p;
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.pos[a] = ST(ZB_S_ROOT_POS + a); p.lv[a] = ST(ZB_S_ROOT_LINVEL + a); p.av[a] = ST(ZB_S_ROOT_ANGVEL + a); }
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = ST(ZB_S_ROOT_QUAT + a);
#pragma unroll
  for (int j = 0; j < ND; ++j) { p.jq[j] = ST(ZB_S_JOINT_POS + j); p.jqd[j] = ST(ZB_S_JOINT_VEL + j); }
  const float* cst = carry_prefetch<ZB_STATE_DIM>(q, st, N, i);
#define CST(f) cst[f]

  // _pre_physics_step (v2.py:276-287); _actions / p_delta are stored with the rest at the end
  // (one writer lane per env; the team holds identical values)
  const bool writer = q.s == 0;
  const float step_dt = cfg.sim_dt * (float)cfg.decimation;
  float target[ND];
  {
    // what the MDP needs after the physics is parked in LDS (Pre), not held in registers
    Pre pr;
    pr.action_rate = 0.f;
    float a_tanh[ND];
    actions_tanh(act, i, q.s, a_tanh);
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float a_prev = ST(ZB_S_ACTIONS + j);
      pr.a_now[j] = a_tanh[j];
      pr.pdel[j] = clampf(ST(ZB_S_P_DELTA + j) + PI_F * pr.a_now[j] * cfg.joint_speed_limit * step_dt, -PI_F, PI_F);
      target[j] = pr.pdel[j] + m->default_joint_pos[j];
      pr.action_rate += (pr.a_now[j] - a_prev) * (pr.a_now[j] - a_prev);   // v2.py:502-507
    }

    // the previous _get_observations cache (one-step lag, v2.py:315-345): the pre-step terms are
    // evaluated now, only what step_length / dones need is carried across the physics
    Cache c;
    wave_sync();  // link table copy
    fk_team_pose(p, q);
    wave_sync();
    make_cache_q(opaque(m), q, p, c);
    pr.r_pre[0] = tanh_r(10.f * c.vfwd / cfg.joint_speed_limit);                     // base_vel_forward
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const float dz[3] = {c.feet_z[f][0], c.feet_z[f][1], c.feet_z[f][2] - 1.f};
      s1 += sqrtf(dot3(dz, dz));                                                 // feet_downward
      const float dx[3] = {c.feet_x[f][0] - c.fwd[0], c.feet_x[f][1] - c.fwd[1], c.feet_x[f][2] - c.fwd[2]};
      s2 += sqrtf(dot3(dx, dx));                                                 // feet_forward
    }
    pr.r_pre[1] = s1;
    pr.r_pre[2] = s2;
    pr.r_pre[3] = fabsf(c.heading_err);                                             // base_heading_x
    pr.r_pre[4] = fabsf(c.feet_pos[0][1] + c.feet_pos[1][1]) + fabsf(c.base_pos[1]); // base_pos_y_err (origin 0)
    pr.base_y = c.base_pos[1];
    pr.base_z = c.base_pos[2];
    pr.heading = c.heading_err;
#pragma unroll
    for (int a = 0; a < 3; ++a) { pr.fwd[a] = c.fwd[a]; pr.feet[0][a] = c.feet_pos[0][a]; pr.feet[1][a] = c.feet_pos[1][a]; }
    if (writer) q.pre() = pr;
  }

  // 4 physics substeps, each followed by the contact sensor's update (record parked in LDS); the
  // last one's applied torques feed the torques term
  SensorOut so;
  wc_load(q, wc, N, i);  // the first substep's GJK warm start (later substeps: the previous one's)
  sp.mark(0);
  for (int k = 0; k < cfg.decimation; ++k) {
    // (a compile-time `true` here lets the scheduler reshape the loop into a 36 B/lane spill)
    substep<false, false, kTgs, kRefresh, kRf>(m, cfg, p, target, q, opaque_true(), true, so, nullptr, nullptr, sp);
    sens_record(q, k, so);
    sp.mark(7);
    sp.substep_end(k);
  }
  m = opaque(m);
  wave_sync();
  const float wc_row = wc_extract(q);
  const Pre pr = q.pre();
  const float(&a_now)[ND] = pr.a_now;
  const float(&pdel)[ND] = pr.pdel;
  const float(&r_pre)[5] = pr.r_pre;
  const float pre_base_y = pr.base_y, pre_base_z = pr.base_z, pre_heading = pr.heading;
  const float(&pre_fwd)[3] = pr.fwd;
  const float(&pre_feet)[2][3] = pr.feet;
  const float r_action_rate = pr.action_rate;

  // MDP state of this env (the LDS carry, or every lane loads; one writer lane stores at the
  // end). The state pointer goes through an empty asm so direct loads are not hoisted above the
  // physics (they would be held in registers across all substeps).
  st = opaque_ptr(st);
  float air_cur[2], air_last[2], contact_t[2], con_last_unused[2] = {0.f, 0.f};
  float step_len[2], f_last0[2], down[2][3], sums0[ZB_NUM_REWARD_TERMS];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    air_cur[f] = CST(ZB_S_FEET_AIR_CUR + f);
    air_last[f] = CST(ZB_S_FEET_AIR_LAST + f);
    contact_t[f] = CST(ZB_S_FEET_CONTACT_CUR + f);
    step_len[f] = CST(ZB_S_FEET_STEP_LEN + f);
    f_last0[f] = CST(ZB_S_FEET_F_LAST + f);
#pragma unroll
    for (int a = 0; a < 3; ++a) down[f][a] = CST(ZB_S_FEET_DOWN_POS + 3 * f + a);
  }
  const float ep_len = CST(ZB_S_EP_LEN) + 1.f;
  const float hs0 = CST(ZB_S_HEADING_SUM), ys0 = CST(ZB_S_Y_ERR_SUM), fs0 = CST(ZB_S_FEET_FORCE_SUM);
#pragma unroll
  for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) sums0[t] = CST(ZB_S_EP_SUMS + t);
  sp.mark(10);

  // ContactSensor (history 5, updated every physics step): histories and timers after the substeps
  float fz_sum[2], fm_max;
  sens_replay<ZB_HIST>(q, cst, 1, 0, ZB_S_FEET_FZ_HIST, ZB_S_UNDES_FMAX_HIST, cfg.decimation, cfg.sim_dt,
                       cfg.contact_force_threshold, fz_sum, fm_max, air_cur, air_last, contact_t, con_last_unused);

  // post-step feet COM velocities (feet_slide); post-step feet positions (the reset latch)
  float feet_vel[2][3], obs_q[4], post_feet[2][3];
  {
    wave_sync();  // the last substep's readers of the body poses are done
    fk_team_pose(p, q);
    wave_sync();
    float S[ND][6], org[ND][3];
    read_joints(q, S, org);
    link_com_vel_q(m, q, p, S, 0, feet_vel[0]);
    link_com_vel_q(m, q, p, S, 11, feet_vel[1]);
    float bp[3], fq[4];
    link_pose_q(m, q, 6, bp, obs_q);  // base quat of the post-step state (observation)
    link_pose_q(m, q, 0, post_feet[0], fq);
    link_pose_q(m, q, 11, post_feet[1], fq);
#pragma unroll
    for (int a = 0; a < 3; ++a) { post_feet[0][a] += p.pos[a]; post_feet[1][a] += p.pos[a]; }
  }
  sp.mark(11);

  // _get_dones (v2.py:384-411)
  const bool time_out = ep_len >= (float)(cfg.max_episode_length - 1);
  float feetF[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) feetF[f] = fz_sum[f] / (float)ZB_HIST;
  bool died = fm_max > 1.0f;
  died |= pre_base_z < cfg.termination_height;
  died |= fabsf(pre_base_y) > 0.5f;  // base_pos_y_err vs env origin (local frame: 0)
  const bool blowup = phys_bad(p);     // non-finite guard (phys_bad)
  died |= blowup;

  // _get_rewards (v2.py:371-382) in dict order. A stateful term's buffers advance only while the
  // term is in the active reward_cfg (they are updated inside its _reward_<name>; cfg.reward_active)
  const uint32_t on = cfg.reward_active;
  float r[ZB_NUM_REWARD_TERMS];
  r[ZB_R_BASE_VEL_FORWARD] = r_pre[0];
  r[ZB_R_FEET_DOWNWARD] = r_pre[1];
  r[ZB_R_FEET_FORWARD] = r_pre[2];
  r[ZB_R_BASE_HEADING_X] = r_pre[3];
  const float hs = (on >> ZB_R_BASE_HEADING_X_SUM) & 1u ? clampf(hs0 + 0.01f * pre_heading, -1.f, 1.f) : hs0;
  r[ZB_R_BASE_HEADING_X_SUM] = fabsf(hs);
  const bool step_on = (on >> ZB_R_STEP_LENGTH) & 1u;
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    if (step_on && feetF[f] > 10.f && f_last0[f] < 10.f) {   // touchdown, v2.py:514-517
      float dv[3];
#pragma unroll
      for (int a = 0; a < 3; ++a) {
        dv[a] = pre_feet[f][a] - down[f][a];
        down[f][a] = pre_feet[f][a];
      }
      step_len[f] = dot3(dv, pre_fwd);
    }
  }
  r[ZB_R_STEP_LENGTH] = tanh_r(15.f * fminf(step_len[0], step_len[1]));
  r[ZB_R_AIRTIME_BALANCE] = fabsf(air_last[0] - air_last[1]);
  r[ZB_R_ACTION_RATE] = r_action_rate;
  r[ZB_R_TORQUES] = so.tau2;
  {
    float sacc = 0.f;
#pragma unroll
    for (int f = 0; f < 2; ++f)
      sacc += sqrtf(feet_vel[f][0] * feet_vel[f][0] + feet_vel[f][1] * feet_vel[f][1]) * (feetF[f] > 1.f ? 1.f : 0.f);
    r[ZB_R_FEET_SLIDE] = sacc;
  }
  r[ZB_R_BASE_POS_Y_ERR] = r_pre[4];
  const float ys = (on >> ZB_R_BASE_POS_Y_ERR_SUM) & 1u ? clampf(ys0 + 0.01f * pre_base_y, -1.f, 1.f) : ys0;
  r[ZB_R_BASE_POS_Y_ERR_SUM] = fabsf(ys);
  r[ZB_R_AIRTIME_SUM] = tanh_r(air_last[0] + air_last[1]);
  // step0's feet-force terms (v2.py:563-571): the difference is signed by the integrator before
  // feet_force_sum updates it (dict order); torch.sign(0) = 0
  r[ZB_R_FEET_FORCE_DIFF] = (feetF[1] - feetF[0]) * (fs0 > 0.f ? 1.f : (fs0 < 0.f ? -1.f : 0.f));
  const float fs = (on >> ZB_R_FEET_FORCE_SUM) & 1u ? fs0 + 0.001f * (feetF[0] - feetF[1]) : fs0;
  r[ZB_R_FEET_FORCE_SUM] = fabsf(fs);

  float reward = 0.f, sums[ZB_NUM_REWARD_TERMS];
  const bool reset = died || time_out;
#pragma unroll
  for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) {
    const float v = r[t] * cfg.reward_scales[t];
    reward += v;
    sums[t] = sums0[t] + v;
  }
  if (died) reward -= cfg.terminal_penalty;  // v2.py:379-380
  if (blowup) {  // finite reward, the episode sums without this step, no carried non-finite latch
    reward = -cfg.terminal_penalty;
#pragma unroll
    for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) sums[t] = sums0[t];
#pragma unroll
    for (int f = 0; f < 2; ++f) { step_len[f] = 0.f; feetF[f] = 0.f; }
  }

  // in-kernel auto-reset (v2.py:413-459): the episode log, then the default state; step_len and
  // f_last are not reset (reference); feet_down_pos_last = the pre-reset (post-step) feet positions
  // (v2.py:436 reads them before sim.forward()), or the default feet with
  // cfg.reset_feet_refresh
  const uint64_t lmask = __ballot(reset && lead);
  if (reset) {
    if (lead) {
      float* lr = log_row(q);
#pragma unroll
      for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) lr[t] = sums[t];   // v2.py:441-448
      lr[ACC_NRES] = 1.f;
      lr[ACC_DIED] = died ? 1.f : 0.f;
      lr[ACC_TOUT] = time_out ? 1.f : 0.f;
    }
#pragma unroll
    for (int a = 0; a < 3; ++a) { p.pos[a] = m->default_root_pos[a]; p.lv[a] = 0.f; p.av[a] = 0.f; }
#pragma unroll
    for (int a = 0; a < 4; ++a) p.quat[a] = m->default_root_quat[a];
#pragma unroll
    for (int j = 0; j < ND; ++j) { p.jq[j] = m->default_joint_pos[j]; p.jqd[j] = 0.f; }
    const float4 d0 = q.dflt()[0], d1 = q.dflt()[1], dq = q.dflt()[2];
    if (cfg.reset_feet_refresh || blowup) {
      down[0][0] = d0.x; down[0][1] = d0.y; down[0][2] = d0.z;
      down[1][0] = d1.x; down[1][1] = d1.y; down[1][2] = d1.z;
    } else {
#pragma unroll
      for (int a = 0; a < 3; ++a) { down[0][a] = post_feet[0][a]; down[1][a] = post_feet[1][a]; }
    }
    obs_q[0] = dq.x; obs_q[1] = dq.y; obs_q[2] = dq.z; obs_q[3] = dq.w;
  }
  log_flush(q, lmask, acc);
  {
    // (an opaque 32-bit index: the load's address is not kept across the physics in a 64-bit register)
    unsigned wi = (unsigned)(q.s * N + i);
    asm volatile("" : "+v"(wi));
    wc[wi] = reset ? wc_invalid(q.s) : wc_row;
  }
  sp.mark(12);
#define OUT(f) q.stg(f)
  if (writer) {
    auto live = [reset](float v) { return reset ? 0.f : v; };  // fields zeroed by _reset_idx
#pragma unroll
    for (int a = 0; a < 3; ++a) { OUT(ZB_S_ROOT_POS + a) = p.pos[a]; OUT(ZB_S_ROOT_LINVEL + a) = p.lv[a]; OUT(ZB_S_ROOT_ANGVEL + a) = p.av[a]; }
#pragma unroll
    for (int a = 0; a < 4; ++a) OUT(ZB_S_ROOT_QUAT + a) = p.quat[a];
#pragma unroll
    for (int j = 0; j < ND; ++j) { OUT(ZB_S_JOINT_POS + j) = p.jq[j]; OUT(ZB_S_JOINT_VEL + j) = p.jqd[j]; }
#pragma unroll
    for (int j = 0; j < ND; ++j) { OUT(ZB_S_P_DELTA + j) = live(pdel[j]); OUT(ZB_S_ACTIONS + j) = live(a_now[j]); }
#pragma unroll
    for (int f = 0; f < 2; ++f) {
#pragma unroll
      for (int a = 0; a < 3; ++a) OUT(ZB_S_FEET_DOWN_POS + 3 * f + a) = down[f][a];
      OUT(ZB_S_FEET_STEP_LEN + f) = step_len[f];
      OUT(ZB_S_FEET_F_LAST + f) = step_on ? feetF[f] : f_last0[f];  // refreshed by step_length only (v2.py:532)
      OUT(ZB_S_FEET_AIR_CUR + f) = live(air_cur[f]);
      OUT(ZB_S_FEET_AIR_LAST + f) = live(air_last[f]);
      OUT(ZB_S_FEET_CONTACT_CUR + f) = live(contact_t[f]);

    }
    sens_store<ZB_HIST>(q, cst, 1, 0, ZB_S_FEET_FZ_HIST, ZB_S_UNDES_FMAX_HIST, cfg.decimation, reset,
                        [&](int row, float v) { OUT(row) = v; });
    OUT(ZB_S_HEADING_SUM) = live(hs);
    OUT(ZB_S_Y_ERR_SUM) = live(ys);
    OUT(ZB_S_FEET_FORCE_SUM) = live(fs);
    OUT(ZB_S_EP_LEN) = live(ep_len);
#pragma unroll
    for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) OUT(ZB_S_EP_SUMS + t) = live(sums[t]);

    // _get_observations (v2.py:351-365) of the post-step / post-reset state
    float* o = &q.stg(ZB_STATE_DIM);
    o[0] = obs_q[0]; o[1] = obs_q[1]; o[2] = obs_q[2]; o[3] = obs_q[3];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      o[4 + j] = p.jq[j] - m->default_joint_pos[j];
      o[10 + j] = p.jqd[j];
      o[16 + j] = live(a_now[j]);
    }
    o[22] = cfg.joint_speed_limit;
    o[ZB_OBS_DIM] = reward;
    o[ZB_OBS_DIM + 1] = died ? 1.f : 0.f;
    o[ZB_OBS_DIM + 2] = time_out ? 1.f : 0.f;
  }
  staged_store<ZB_STATE_DIM, ZB_OBS_DIM>(q, xcd_block(blockIdx.x, gridDim.x) * EPW, N, st, obs, rew, term, trunc, done);
#undef OUT
  sp.mark(8);
  sp.flush();
#undef ST
#undef CST
}

// kOcc (every step kernel): 2 = up to 256 registers (two waves per SIMD once a launch has more
// waves than SIMDs); 1 = 512 registers (256 VGPRs + 256 AGPRs claimed), so one wave per SIMD: at
// N <= 4096 envs (<= 1024 waves) the dispatcher then gives every wave its own SIMD, whereas with
// two-wave occupancy it doubles up 6-11 % of the SIMDs and leaves as many idle
// (tools/probe/wave_placement.hip), and the doubled-up waves set the launch's tail.
// kRf: the ruling-on-face manifold compiled in (launched for self_manifold 3 only)
template <bool kTgs, int kOcc, bool kRefresh = false, bool kRf = false>
__global__ __launch_bounds__(WGT, kOcc) void zb_step_kernel(const zb_model* __restrict__ mg,
                                                          const float4* __restrict__ links, zb_task_cfg cfg, int N,
                                                          float* __restrict__ st, const float* __restrict__ act,
                                                          float* __restrict__ obs, float* __restrict__ rew,
                                                          uint8_t* __restrict__ term, uint8_t* __restrict__ trunc,
                                                          int64_t* __restrict__ done, float* __restrict__ acc,
                                                          float* __restrict__ wc) {
  __shared__ float4 lds[LDS4];
  if (kOcc == 1) asm volatile("" ::: "a255");
  step_body<kTgs, kRefresh, kRf>(mg, links, cfg, N, st, act, obs, rew, term, trunc, done, acc, wc, lds);
}

// Test entry (zb_pair_manifold): GJK (cold start) + the face manifold of n link pairs given as
// world-frame core hulls, one pair per quad (tests/test_gpu_selfcollision.py against the oracle's
// zbo_pair_manifold): out [n][29] = {points, then per point {sep, n[3], x[3]}} (0 points: no contact;
// 1 without a face manifold: the GJK contact).
__global__ void zb_manifold_kernel(const float* __restrict__ pairs, int n, float margin, int mode, float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int pr = min(t >> 2, n - 1), j = t & 3;  // quads past n recompute pair n - 1 (no store)
  const float* c = pairs + (size_t)pr * 36 + 9 * j;
  QCircle h;
#pragma unroll
  for (int k = 0; k < 3; ++k) { h.c[k] = c[k]; h.e1[k] = c[3 + k]; h.e2[k] = c[6 + k]; }
  float ca[3], cb[3], v0[3];
  quad_centres(h, ca, cb);
  v0[0] = ca[0] - cb[0]; v0[1] = ca[1] - cb[1]; v0[2] = ca[2] - cb[2];
  SelfContact sc;
  int its = 0;
  const bool hit = gjk_quad(h, j, v0, false, margin, margin, sc, its);
  float* o = out + (size_t)pr * 29;
  const bool mine = (t >> 2) < n;
  int cnt = 0;
  if (hit && sc.sep > -2.f * kCoreM + 1e-7f)
    cnt = quad_manifold<true>(h, j, sc, margin, true, mode, [&](int rank, float4 xs, const float* nn) {
      if (mine) {
        float* p = o + 1 + 7 * rank;
        p[0] = xs.w; p[1] = nn[0]; p[2] = nn[1]; p[3] = nn[2]; p[4] = xs.x; p[5] = xs.y; p[6] = xs.z;
      }
    });
  if (mine && j == 0) {
    if (hit && cnt == 0) {
      float* p = o + 1;
      p[0] = sc.sep; p[1] = sc.n[0]; p[2] = sc.n[1]; p[3] = sc.n[2]; p[4] = sc.x[0]; p[5] = sc.x[1]; p[6] = sc.x[2];
    }
    o[0] = hit ? (float)(cnt > 0 ? cnt : 1) : 0.f;
  }
}

// Test entry (zb_gjk_pairs): the self-collision GJK of n link pairs given as world-frame core
// hulls, one pair per quad (tests/test_gpu_selfcollision.py against the oracle's hull_pair).
// pairs: [n][2 hulls][2 circles][9] (centre, E1, E2; radius baked in); v0: [n][3] start
// directions or NULL (hull centre difference); out: [n][9] {contact, sep, n[3], x[3], iterations}.
__global__ void zb_gjk_kernel(const float* __restrict__ pairs, const float* __restrict__ v0s, int n, float margin,
                              float* __restrict__ out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int pr = min(t >> 2, n - 1), j = t & 3;  // quads past n recompute pair n - 1 (no store)
  const float* c = pairs + (size_t)pr * 36 + 9 * j;
  QCircle h;
#pragma unroll
  for (int k = 0; k < 3; ++k) { h.c[k] = c[k]; h.e1[k] = c[3 + k]; h.e2[k] = c[6 + k]; }
  float v0[3];
  {
    float ca[3], cb[3];
    quad_centres(h, ca, cb);
    v0[0] = ca[0] - cb[0]; v0[1] = ca[1] - cb[1]; v0[2] = ca[2] - cb[2];
  }
  if (v0s)
    for (int k = 0; k < 3; ++k) v0[k] = v0s[(size_t)pr * 3 + k];
  SelfContact sc = {};
  int its = 0;
  const bool hit = gjk_quad(h, j, v0, v0s != nullptr, margin, margin, sc, its);
  if (j == 0 && (t >> 2) < n) {
    float* o = out + (size_t)pr * 9;
    o[0] = hit ? 1.f : 0.f;
    o[1] = sc.sep;
    for (int k = 0; k < 3; ++k) { o[2 + k] = sc.n[k]; o[5 + k] = sc.x[k]; }
    o[8] = (float)its;
  }
}

// reset env_ids (or all when ids == nullptr); logs the reset envs' episode sums into acc
__global__ void zb_reset_kernel(const zb_model* __restrict__ mg, const float4* __restrict__ links, int N,
                                float* __restrict__ st, const int32_t* __restrict__ ids, int n,
                                float* __restrict__ acc, int refresh) {
  MP m = to_mp(mg);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int i = ids ? ids[t] : t;
  if (i < 0 || i >= N) return;
  Phys p;
  Mdp d;
  load_state(st, N, i, p, d);
#pragma unroll
  for (int k = 0; k < ZB_NUM_REWARD_TERMS; ++k) atomicAdd(&acc_slot(acc, t)[k], d.sums[k]);
  atomicAdd(&acc_slot(acc, t)[ACC_NRES], 1.f);
  reset_env(m, links + DFLT_OFF, p, d, refresh);
  store_state(st, N, i, p, d);
}

// default-pose constants for resets (once, at zb_create): feet link positions and the base
// link quaternion of the default root pose / joint positions
__global__ void zb_derive_kernel(const zb_model* __restrict__ mg, float4* __restrict__ links) {
  MP m = to_mp(mg);
  Phys p;
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.pos[a] = m->default_root_pos[a]; p.lv[a] = 0.f; p.av[a] = 0.f; }
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = m->default_root_quat[a];
#pragma unroll
  for (int j = 0; j < ND; ++j) { p.jq[j] = m->default_joint_pos[j]; p.jqd[j] = 0.f; }
  Kin k;
  fk(m, p, k);
  float f0[3], f1[3], bp[3], q0[4];
  link_pose(m, k, m->foot_links[0], f0, q0);
  link_pose(m, k, m->foot_links[1], f1, q0);
  link_pose(m, k, m->base_link, bp, q0);
  links[DFLT_OFF + 0] = make_float4(f0[0] + p.pos[0], f0[1] + p.pos[1], f0[2] + p.pos[2], 0.f);
  links[DFLT_OFF + 1] = make_float4(f1[0] + p.pos[0], f1[1] + p.pos[1], f1[2] + p.pos[2], 0.f);
  links[DFLT_OFF + 2] = make_float4(q0[0], q0[1], q0[2], q0[3]);
  // base link orientation relative to the root at the default joint positions
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = a == 0 ? 1.f : 0.f;
#pragma unroll
  for (int a = 0; a < 3; ++a) p.pos[a] = 0.f;
  fk(m, p, k);
  link_pose(m, k, m->base_link, bp, q0);
  links[DFLT_OFF + 3] = make_float4(q0[0], q0[1], q0[2], q0[3]);
  link_pose(m, k, m->foot_links[0], f0, q0);
  link_pose(m, k, m->foot_links[1], f1, q0);
  links[DFLT_OFF + 4] = make_float4(f0[0], f0[1], f0[2], 0.f);
  links[DFLT_OFF + 5] = make_float4(f1[0], f1[1], f1[2], 0.f);
}

__global__ void zb_observe_kernel(const zb_model* __restrict__ mg, int N, const float* __restrict__ st,
                                  float* __restrict__ obs) {
  MP m = to_mp(mg);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  Phys p;
  Mdp d;
  load_state(st, N, i, p, d);
  write_obs(m, p, d, obs, i);
}

template <bool kLinkFriction, bool kTgs, bool kRefresh = false>
__global__ __launch_bounds__(WGT, ZB_WAVES_PER_SIMD) void zb_substeps_kernel(const zb_model* __restrict__ mg,
                                                              const float4* __restrict__ links, zb_task_cfg cfg, int N,
                                                              float* __restrict__ st, const float* __restrict__ targets,
                                                              int nsub, float* __restrict__ net_force,
                                                              float* __restrict__ tau_out) {
  MP m = to_mp(mg);
  __shared__ float4 lds[LDS4];
  const int lane = threadIdx.x;
  const int env = xcd_block(blockIdx.x, gridDim.x) * EPW + lane / TL;
  const int i = env < N ? env : N - 1;
  const Q q = make_q(lds, lane, links);
  for (int t = LNK_G + lane; t < LNK4; t += WGT) lds[LNK_OFF + t] = links[t];
  const int mu_row = cfg.task == ZB_TASK_MANAGER_V0 ? ZB_M_LINK_MU : ZB_SU_LINK_MU;
  const int mud_row = cfg.task == ZB_TASK_MANAGER_V0 ? ZB_M_LINK_MU_D : ZB_SU_LINK_MU_D;
  if (kLinkFriction && q.s < NL) {
    q.fric(q.s) = st[(size_t)(mu_row + q.s) * N + i];
    q.fricd(q.s) = st[(size_t)(mud_row + q.s) * N + i];
  }
  Phys p;
  load_phys(st, N, i, p);
  float tg[ND], tau[ND], F[1][3];
#pragma unroll
  for (int j = 0; j < ND; ++j) { tg[j] = targets[(size_t)i * ND + j]; tau[j] = 0.f; }
  SensorOut so;
  Stamps sp;
  for (int k = 0; k < nsub; ++k)
    substep<true, kLinkFriction, kTgs, kRefresh, true>(m, cfg, p, tg, q, k == nsub - 1, k > 0, so, F, tau, sp);
  if (net_force && q.s < NL)
#pragma unroll
    for (int a = 0; a < 3; ++a) net_force[((size_t)i * NL + q.s) * 3 + a] = F[0][a];
  if (tau_out)
#pragma unroll
    for (int j = 0; j < ND; ++j) tau_out[(size_t)i * ND + j] = tau[j];
#define SV(f, v) st[(size_t)(f) * N + i] = (v)
#pragma unroll
  for (int a = 0; a < 3; ++a) { SV(ZB_S_ROOT_POS + a, p.pos[a]); SV(ZB_S_ROOT_LINVEL + a, p.lv[a]); SV(ZB_S_ROOT_ANGVEL + a, p.av[a]); }
#pragma unroll
  for (int a = 0; a < 4; ++a) SV(ZB_S_ROOT_QUAT + a, p.quat[a]);
#pragma unroll
  for (int j = 0; j < ND; ++j) { SV(ZB_S_JOINT_POS + j, p.jq[j]); SV(ZB_S_JOINT_VEL + j, p.jqd[j]); }
#undef SV
}


// =========================================================================== stand-up task
// zbot-6b-standup-v0 (reference zbot_direct_6_standup_env_v0.py = standup.py) on the same robot
// and physics: ZBOT_6S_CFG_2 lying init (zbot_cfg.py:721-763), per-link friction from the
// startup material randomisation, rewards from the post-step link states, died on a height drop,
// reset pose randomised in-kernel (reset_root_state_uniform) and a device-side curriculum.

__host__ __device__ __forceinline__ float u01(uint64_t h) { return (float)(h >> 40) * (1.0f / 16777216.0f); }

// reward weight of term t in curriculum stage `stage` (compile-time indices into the kernarg table)
__device__ __forceinline__ float stage_weight(const zb_task_cfg& cfg, int stage, int t) {
  float w = cfg.stage_scales[0][t];
#pragma unroll
  for (int sg = 1; sg < ZB_MAX_STAGES; ++sg) w = stage == sg ? cfg.stage_scales[sg][t] : w;
  return w;
}

// counter-based random stream of env i at call ctr; draw k of it (shared with the oracle)
__device__ __forceinline__ uint64_t env_hash(uint64_t seed, uint64_t ctr, int i) {
  return hash64(seed ^ hash64(ctr * 0x100000001B3ull + (uint64_t)i));
}
__device__ __forceinline__ float draw(uint64_t h, int k) { return u01(hash64(h + 0x632BE59BD9B4E019ull * (uint64_t)k)); }

// reset_root_state_uniform (standup.py:33-97, v4.py:59-105) from stream h (draws 1..4): x, y,
// roll, yaw ~ U (the cfg ranges; pitch / z / velocities 0), root = default + (x, y, 0), quat =
// quat_from_euler_xyz(roll, 0, yaw) applied in the world frame (delta * default, standup) or the
// body frame (default * delta, v4), normalised; joints default, every velocity zero. Returns the
// yaw sample (the events store it as env.current_yaw).
__device__ __forceinline__ float reset_pose(MP m, const zb_task_cfg& cfg, uint64_t h, Phys& p) {
  float r[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    r[k] = draw(h, k + 1) * (cfg.reset_pose_range[k][1] - cfg.reset_pose_range[k][0]) + cfg.reset_pose_range[k][0];
  float sr, cr, sy, cy;
  sincos_r(0.5f * r[2], &sr, &cr);
  sincos_r(0.5f * r[3], &sy, &cy);
  const float dq[4] = {cy * cr, cy * sr, sy * sr, sy * cr};  // quat_from_euler_xyz(roll, 0, yaw)
  // the sampled pose is the Isaac Lab root's (the chain root unless the asset is rooted elsewhere):
  // its default pose is chain-root default * T (T = api_root_in_root, identity for the others)
  const float q0[4] = {m->default_root_quat[0], m->default_root_quat[1], m->default_root_quat[2],
                       m->default_root_quat[3]};
  const float tT[3] = {m->api_root_in_root[0], m->api_root_in_root[1], m->api_root_in_root[2]};
  const float qT[4] = {m->api_root_in_root[3], m->api_root_in_root[4], m->api_root_in_root[5], m->api_root_in_root[6]};
  float qa0[4], ta[3];
  qmul(q0, qT, qa0);
  qrot(q0, tT, ta);
  float qa[4];
  if (cfg.reset_pose_body_frame) qmul(qa0, dq, qa);
  else qmul(dq, qa0, qa);
  qnormalize(qa);
  const float pa[3] = {m->default_root_pos[0] + ta[0] + r[0], m->default_root_pos[1] + ta[1] + r[1],
                       m->default_root_pos[2] + ta[2]};
  // back to the chain root: q = qa * conj(qT), p = pa - R(q) tT
  const float qTc[4] = {qT[0], -qT[1], -qT[2], -qT[3]};
  float qn[4], tq[3];
  qmul(qa, qTc, qn);
  qrot(qn, tT, tq);
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = qn[a];
  p.pos[0] = pa[0] - tq[0];
  p.pos[1] = pa[1] - tq[1];
  p.pos[2] = pa[2] - tq[2];
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.lv[a] = 0.f; p.av[a] = 0.f; }
#pragma unroll
  for (int j = 0; j < ND; ++j) { p.jq[j] = m->default_joint_pos[j]; p.jqd[j] = 0.f; }
  return r[3];
}

__device__ __forceinline__ void su_reset_pose(MP m, const zb_task_cfg& cfg, uint64_t seed, uint64_t ctr, int i,
                                              Phys& p) {
  (void)reset_pose(m, cfg, env_hash(seed, ctr, i), p);
}

// One stand-up policy step per team (same mapping as zb_step_kernel; no contact sensor).
template <bool kTgs, int kOcc, bool kRefresh = false, bool kRf = false>
__global__ __launch_bounds__(WGT, kOcc) void zb_su_step_kernel(
    const zb_model* __restrict__ mg, const float4* __restrict__ links, zb_task_cfg cfg, int N, float* __restrict__ st,
    const float* __restrict__ act, float* __restrict__ obs, float* __restrict__ rew, uint8_t* __restrict__ term,
    uint8_t* __restrict__ trunc, int64_t* __restrict__ done, float* __restrict__ acc,
    const Counters* __restrict__ cnt, uint64_t seed, float* __restrict__ wc) {
  MP m = to_mp(mg);
  __shared__ float4 lds[LDS4];
  if (kOcc == 1) asm volatile("" ::: "a255");  // (zb_step_kernel: kOcc)
  const int lane = threadIdx.x;
  const int env = xcd_block(blockIdx.x, gridDim.x) * EPW + lane / TL;
  const int i = env < N ? env : N - 1;
  const bool lead = env < N && lane % TL == 0;
  const Q q = make_q(lds, lane, links);
  for (int t = LNK_G + lane; t < LNK4; t += WGT) lds[LNK_OFF + t] = links[t];
  Stamps sp;
  sp.begin();
#define ST(f) st[(size_t)(f) * N + i]
  Phys p;
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.pos[a] = ST(ZB_S_ROOT_POS + a); p.lv[a] = ST(ZB_S_ROOT_LINVEL + a); p.av[a] = ST(ZB_S_ROOT_ANGVEL + a); }
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = ST(ZB_S_ROOT_QUAT + a);
#pragma unroll
  for (int j = 0; j < ND; ++j) { p.jq[j] = ST(ZB_S_JOINT_POS + j); p.jqd[j] = ST(ZB_S_JOINT_VEL + j); }
  if (q.s < NL) {  // lane l: link l (visible after the first barrier)
    q.fric(q.s) = ST(ZB_SU_LINK_MU + q.s);
    q.fricd(q.s) = ST(ZB_SU_LINK_MU_D + q.s);
  }

  // _pre_physics_step (standup.py:538-551, mode 1)
  const bool writer = q.s == 0;
  const float step_dt = cfg.sim_dt * (float)cfg.decimation;
  float target[ND];
  {
    Pre pr;
    float a_tanh[ND];
    actions_tanh(act, i, q.s, a_tanh);
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      pr.a_now[j] = a_tanh[j];
      pr.pdel[j] = clampf(ST(ZB_SU_P_DELTA + j) + PI_F * pr.a_now[j] * cfg.joint_speed_limit * step_dt, -PI_F, PI_F);
      target[j] = pr.pdel[j] + m->default_joint_pos[j];
    }
    if (writer) q.pre() = pr;
  }

  SensorOut so;
  wc_load(q, wc, N, i);  // the first substep's GJK warm start
  sp.mark(0);
  for (int k = 0; k < cfg.decimation; ++k) {
    substep<false, true, kTgs, kRefresh, kRf>(m, cfg, p, target, q, false, true, so, nullptr, nullptr, sp);
    sp.mark(7);
  }
  m = opaque(m);
  wave_sync();
  const float wc_row = wc_extract(q);
  const Pre pr = q.pre();
  st = opaque_ptr(st);
  const float czl0 = ST(ZB_SU_CENTER_Z_LAST);
  const float ep_len = ST(ZB_SU_EP_LEN) + 1.f;
  float sums0[ZB_SU_NUM_REWARD_TERMS];
#pragma unroll
  for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) sums0[t] = ST(ZB_SU_EP_SUMS + t);
  const int stage = cnt->stage;

  // post-step link states (_compute_intermediate_values 571-591, body_link_state_w)
  float z4, z6, z8, vz5, vz6, fz[2][3], obs_q[4];
  {
    wave_sync();
    fk_team_pose(p, q);
    wave_sync();
    float S[ND][6], org[ND][3];
    read_joints(q, S, org);
    float lp[3], lq[4], v[3], R[9];
    link_pose_q(m, q, 4, lp, lq);
    z4 = lp[2] + p.pos[2];
    link_pose_q(m, q, 8, lp, lq);
    z8 = lp[2] + p.pos[2];
    link_pose_q(m, q, 6, lp, obs_q);
    z6 = lp[2] + p.pos[2];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      link_pose_q(m, q, f == 0 ? 0 : 11, lp, lq);
      qmat(lq, R);
      const float sg = f == 0 ? 1.f : -1.f;  // axis_z_feet = (0,0,1), (0,0,-1) (standup.py:503-505)
      fz[f][0] = sg * R[2]; fz[f][1] = sg * R[5]; fz[f][2] = sg * R[8];
    }
    link_origin_vel_q(m, q, p, S, 6, v);
    vz6 = v[2];
    link_origin_vel_q(m, q, p, S, 5, v);
    vz5 = v[2];
  }

  // _get_dones (standup.py:634-643)
  const bool time_out = ep_len >= (float)(cfg.max_episode_length - 1);
  const bool blowup = phys_bad(p);  // non-finite guard (phys_bad)
  const bool died = (czl0 - z6) > cfg.center_z_drop || blowup;
  const float czl = ((int)ep_len % cfg.center_z_period == cfg.center_z_period - 1) ? z6 : czl0;

  // _get_rewards (standup.py:620-632): reward_func() * scale * step_dt per term, dict order
  float r[ZB_SU_NUM_REWARD_TERMS];
  {
    const float rh = z6 + 0.5f * z4 + 0.5f * z8 - 0.1f;  // _reward_upward_2 (843-856)
    float up = z6 < 0.22f ? rh + 0.5f * vz6 + 0.5f * vz5 : 1.35f;
    if ((fz[0][2] < 0.5f || fz[1][2] < 0.5f) && z6 > 0.1f) up = -5.f * up;
    r[ZB_SU_R_UPWARD_2] = up;
  }
  r[ZB_SU_R_SHAPE_SYMMETRY] = fabsf(pr.pdel[0] + pr.pdel[5]) + fabsf(pr.pdel[1] + pr.pdel[4]) +
                              fabsf(pr.pdel[2] + pr.pdel[3]);  // 782-789
  {
    float sd = 0.f;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const float d[3] = {fz[f][0], fz[f][1], fz[f][2] - 1.f};
      sd += sqrtf(dot3(d, d));
    }
    r[ZB_SU_R_FEET_DOWNWARD] = sd;  // 735-745
  }
  r[ZB_SU_R_FEET_DOWNWARD_4] = z6 < 0.15f ? fz[0][2] + fz[1][2] : 1.6f;  // 827-840
  float w[ZB_SU_NUM_REWARD_TERMS];
#pragma unroll
  for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) w[t] = stage_weight(cfg, stage, t);
  float reward = 0.f, sums[ZB_SU_NUM_REWARD_TERMS];
#pragma unroll
  for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) {
    const float v = (r[t] * w[t]) * step_dt;
    reward += v;
    sums[t] = sums0[t] + v;
  }
  if (died) reward -= cfg.terminal_penalty;  // 629-630
  if (blowup) {
    reward = -cfg.terminal_penalty;
#pragma unroll
    for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) sums[t] = sums0[t];
  }
  const bool reset = died || time_out;

  // _reset_idx (645-703): episode log (sums per second of the env's own episode), new random
  // root pose, default joints; the reset env's observation sees the new pose
  const uint64_t lmask = __ballot(reset && lead);
  if (reset) {
    if (lead) {
      const float dur = fmaxf(ep_len * step_dt, step_dt);
      float* lr = log_row(q);
#pragma unroll
      for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) lr[t] = sums[t] / dur;
      lr[ACC_NRES] = 1.f;
      lr[ACC_DIED] = died ? 1.f : 0.f;
      lr[ACC_TOUT] = time_out ? 1.f : 0.f;
    }
    su_reset_pose(m, cfg, seed, cnt->calls, i, p);
    const float4 qr = q.dflt()[3];
    const float qrel[4] = {qr.x, qr.y, qr.z, qr.w};
    qmul(p.quat, qrel, obs_q);
  }
  log_flush(q, lmask, acc);
  {
    // (an opaque 32-bit index: the load's address is not kept across the physics in a 64-bit register)
    unsigned wi = (unsigned)(q.s * N + i);
    asm volatile("" : "+v"(wi));
    wc[wi] = reset ? wc_invalid(q.s) : wc_row;
  }
  sp.mark(12);
#define OUT(f) q.stg(f)
  if (writer) {
    auto live = [reset](float v) { return reset ? 0.f : v; };
#pragma unroll
    for (int a = 0; a < 3; ++a) { OUT(ZB_S_ROOT_POS + a) = p.pos[a]; OUT(ZB_S_ROOT_LINVEL + a) = p.lv[a]; OUT(ZB_S_ROOT_ANGVEL + a) = p.av[a]; }
#pragma unroll
    for (int a = 0; a < 4; ++a) OUT(ZB_S_ROOT_QUAT + a) = p.quat[a];
#pragma unroll
    for (int j = 0; j < ND; ++j) { OUT(ZB_S_JOINT_POS + j) = p.jq[j]; OUT(ZB_S_JOINT_VEL + j) = p.jqd[j]; }
#pragma unroll
    for (int j = 0; j < ND; ++j) { OUT(ZB_SU_P_DELTA + j) = live(pr.pdel[j]); OUT(ZB_SU_ACTIONS + j) = live(pr.a_now[j]); }
    OUT(ZB_SU_CENTER_Z_LAST) = reset ? cfg.center_z_init : czl;
    OUT(ZB_SU_EP_LEN) = live(ep_len);
#pragma unroll
    for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) OUT(ZB_SU_EP_SUMS + t) = live(sums[t]);

    // _get_observations (593-618): base quat, joint_pos - default, joint_vel, actions
    float* o = &q.stg(ZB_SU_LINK_MU);
    o[0] = obs_q[0]; o[1] = obs_q[1]; o[2] = obs_q[2]; o[3] = obs_q[3];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      o[4 + j] = p.jq[j] - m->default_joint_pos[j];
      o[10 + j] = p.jqd[j];
      o[16 + j] = live(pr.a_now[j]);
    }
    q.stg(ZB_SU_LINK_MU + ZB_SU_OBS_DIM) = reward;
    q.stg(ZB_SU_LINK_MU + ZB_SU_OBS_DIM + 1) = died ? 1.f : 0.f;
    q.stg(ZB_SU_LINK_MU + ZB_SU_OBS_DIM + 2) = time_out ? 1.f : 0.f;
  }
  staged_store<ZB_SU_LINK_MU, ZB_SU_OBS_DIM>(q, xcd_block(blockIdx.x, gridDim.x) * EPW, N, st, obs, rew, term, trunc, done);
#undef OUT
  sp.mark(8);
  sp.flush();
#undef ST
}

// explicit resets (env_ids, or all when ids == nullptr): episode log into acc, then the reset
// pose of su_reset_pose; one thread per env
__global__ void zb_su_reset_kernel(const zb_model* __restrict__ mg, zb_task_cfg cfg, int N, float* __restrict__ st,
                                   const int32_t* __restrict__ ids, int n, float* __restrict__ acc,
                                   const Counters* __restrict__ cnt, uint64_t seed) {
  MP m = to_mp(mg);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int i = ids ? ids[t] : t;
  if (i < 0 || i >= N) return;
#define ST(f) st[(size_t)(f) * N + i]
  const float step_dt = cfg.sim_dt * (float)cfg.decimation;
  const float dur = fmaxf(ST(ZB_SU_EP_LEN) * step_dt, step_dt);
#pragma unroll
  for (int k = 0; k < ZB_SU_NUM_REWARD_TERMS; ++k) atomicAdd(&acc_slot(acc, t)[k], ST(ZB_SU_EP_SUMS + k) / dur);
  atomicAdd(&acc_slot(acc, t)[ACC_NRES], 1.f);
  Phys p;
  su_reset_pose(m, cfg, seed, cnt->calls, i, p);
#pragma unroll
  for (int a = 0; a < 3; ++a) { ST(ZB_S_ROOT_POS + a) = p.pos[a]; ST(ZB_S_ROOT_LINVEL + a) = p.lv[a]; ST(ZB_S_ROOT_ANGVEL + a) = p.av[a]; }
#pragma unroll
  for (int a = 0; a < 4; ++a) ST(ZB_S_ROOT_QUAT + a) = p.quat[a];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    ST(ZB_S_JOINT_POS + j) = p.jq[j]; ST(ZB_S_JOINT_VEL + j) = p.jqd[j];
    ST(ZB_SU_P_DELTA + j) = 0.f; ST(ZB_SU_ACTIONS + j) = 0.f;
  }
  ST(ZB_SU_CENTER_Z_LAST) = cfg.center_z_init;
  ST(ZB_SU_EP_LEN) = 0.f;
#pragma unroll
  for (int k = 0; k < ZB_SU_NUM_REWARD_TERMS; ++k) ST(ZB_SU_EP_SUMS + k) = 0.f;
#undef ST
}

__global__ void zb_su_observe_kernel(const zb_model* __restrict__ mg, int N, const float* __restrict__ st,
                                     float* __restrict__ obs) {
  MP m = to_mp(mg);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  Phys p;
  load_phys(st, N, i, p);
  Kin k;
  fk(m, p, k);
  float bp[3], bq[4];
  link_pose(m, k, 6, bp, bq);
  float* o = obs + (size_t)i * ZB_SU_OBS_DIM;
  o[0] = bq[0]; o[1] = bq[1]; o[2] = bq[2]; o[3] = bq[3];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    o[4 + j] = p.jq[j] - m->default_joint_pos[j];
    o[10 + j] = p.jqd[j];
    o[16 + j] = st[(size_t)(ZB_SU_ACTIONS + j) * N + i];
  }
}

// per-link friction [N][NL] -> state rows ZB_SU_LINK_MU (mu == nullptr: fill with `fill`)
__global__ void zb_su_friction_kernel(int N, float* __restrict__ st, const float* __restrict__ mu, float fill, int row) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= N * NL) return;
  const int i = t / NL, l = t % NL;
  st[(size_t)(row + l) * N + i] = mu ? mu[t] : fill;
}

// =========================================================================== walking v4
// zbot-6b-walking-v4 (reference zbot_direct_6dof_bipedal_env_v4.py = v4.py): v2's robot and
// physics with forward-velocity / heading commands (reset and interval resample events), a
// history-3 contact sensor that also tracks contact time, 15 reward terms evaluated on the
// post-step state, and the two curricula (stage weights + command ranges in the device counters).

__device__ __forceinline__ float wrap_to_pi(float x) {  // isaaclab.utils.math.wrap_to_pi
  float a = fmodf(x, TWO_PI_F);
  if (a < 0.f) a += TWO_PI_F;
  return a > PI_F ? a - TWO_PI_F : a;
}

// resample_commands (v4.py:107-135) from stream h, draws k0 .. k0+2, with the device-side params
__device__ __forceinline__ void v4_resample(const zb_task_cfg& cfg, const Counters* cnt, uint64_t h, int k0,
                                            float cur_yaw, float cmd[2], float& target) {
  const float lo = cnt->vel[0], hi0 = cnt->vel[1];
  if (cfg.cmd_dual_sign) {
    const float sg = draw(h, k0) < cnt->prob_pos ? 1.f : -1.f;  // bernoulli(prob_pos) * 2 - 1
    const float hi = hi0 + cfg.cmd_offset * (sg - 1.f);
    cmd[0] = (draw(h, k0 + 1) * (hi - lo) + lo) * sg;
  } else {
    cmd[0] = draw(h, k0 + 1) * (hi0 - lo) + lo;
  }
  cmd[1] = draw(h, k0 + 2) * (cnt->yaw[1] - cnt->yaw[0]) + cnt->yaw[0];
  target = wrap_to_pi(cur_yaw + cmd[1]);
}

// prologue values parked in LDS across the physics (overlays the Pre record)
struct PreV4 {
  float a_now[ND], pdel[ND], jqd_prev[ND], action_rate;
};
static_assert(sizeof(PreV4) <= 16 * PRE4, "PreV4 fits PRE4 granules");

template <bool kTgs, int kOcc>
__global__ __launch_bounds__(WGT, kOcc) void zb_v4_step_kernel(
    const zb_model* __restrict__ mg, const float4* __restrict__ links, zb_task_cfg cfg, int N, float* __restrict__ st,
    const float* __restrict__ act, float* __restrict__ obs, float* __restrict__ rew, uint8_t* __restrict__ term,
    uint8_t* __restrict__ trunc, int64_t* __restrict__ done, float* __restrict__ acc,
    const Counters* __restrict__ cnt, uint64_t seed, float* __restrict__ wc) {
  MP m = to_mp(mg);
  __shared__ float4 lds[LDS4];
  if (kOcc == 1) asm volatile("" ::: "a255");  // (zb_step_kernel: kOcc)
  const int lane = threadIdx.x;
  const int env = xcd_block(blockIdx.x, gridDim.x) * EPW + lane / TL;
  const int i = env < N ? env : N - 1;
  const bool lead = env < N && lane % TL == 0;
  const Q q = make_q(lds, lane, links);
  for (int t = LNK_G + lane; t < LNK4; t += WGT) lds[LNK_OFF + t] = links[t];
  Stamps sp;
  sp.begin();
#define ST(f) st[(size_t)(f) * N + i]
  Phys p;
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.pos[a] = ST(ZB_S_ROOT_POS + a); p.lv[a] = ST(ZB_S_ROOT_LINVEL + a); p.av[a] = ST(ZB_S_ROOT_ANGVEL + a); }
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = ST(ZB_S_ROOT_QUAT + a);
#pragma unroll
  for (int j = 0; j < ND; ++j) { p.jq[j] = ST(ZB_S_JOINT_POS + j); p.jqd[j] = ST(ZB_S_JOINT_VEL + j); }
  const float* cst = carry_prefetch<ZB_V4_STATE_DIM>(q, st, N, i);
#define CST(f) cst[f]

  // _pre_physics_step (v4.py:776-804, mode 1)
  const bool writer = q.s == 0;
  const float step_dt = cfg.sim_dt * (float)cfg.decimation;
  PreV4& pv = *reinterpret_cast<PreV4*>(&q.pre());
  float target[ND];
  {
    PreV4 pr;
    pr.action_rate = 0.f;
    float a_tanh[ND];
    actions_tanh(act, i, q.s, a_tanh);
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float a_prev = ST(ZB_V4_ACTIONS + j);
      pr.a_now[j] = a_tanh[j];
      pr.pdel[j] = clampf(ST(ZB_V4_P_DELTA + j) + PI_F * pr.a_now[j] * cfg.joint_speed_limit * step_dt, -PI_F, PI_F);
      target[j] = pr.pdel[j] + m->default_joint_pos[j];
      pr.action_rate += (pr.a_now[j] - a_prev) * (pr.a_now[j] - a_prev);
      pr.jqd_prev[j] = 0.f;
    }
    if (writer) pv = pr;
  }

  // 4 substeps, each followed by the contact sensor's update (record parked in LDS); the last one's
  // applied torques feed the torques term, the joint velocities before it give Isaac Lab's
  // finite-difference joint_acc (ArticulationData.update every substep)
  SensorOut so;
  wc_load(q, wc, N, i);  // the first substep's GJK warm start
  sp.mark(0);
  for (int k = 0; k < cfg.decimation; ++k) {
    const bool last = k == cfg.decimation - 1;
    if (last && writer) {
#pragma unroll
      for (int j = 0; j < ND; ++j) pv.jqd_prev[j] = p.jqd[j];
    }
    substep<false, false, kTgs>(m, cfg, p, target, q, true, true, so, nullptr, nullptr, sp);
    sens_record(q, k, so);
    sp.mark(7);
  }
  m = opaque(m);
  wave_sync();
  const float wc_row = wc_extract(q);
  const PreV4 pr = pv;
  st = opaque_ptr(st);

  // ContactSensor (history 3, updated every physics step; air / contact timers incl.
  // last_contact_time)
  float fz_sum[2], fm_max;
  float air_cur[2], con_cur[2], air_last[2], con_last[2], feetF[2];
  bool in_contact[2];
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    air_cur[f] = CST(ZB_V4_FEET_AIR_CUR + f);
    con_cur[f] = CST(ZB_V4_FEET_CONTACT_CUR + f);
    air_last[f] = CST(ZB_V4_FEET_AIR_LAST + f);
    con_last[f] = CST(ZB_V4_FEET_CONTACT_LAST + f);
  }
  sens_replay<ZB_V4_HIST>(q, cst, 1, 0, ZB_V4_FEET_FZ_HIST, ZB_V4_UNDES_FMAX_HIST, cfg.decimation, cfg.sim_dt,
                          cfg.contact_force_threshold, fz_sum, fm_max, air_cur, air_last, con_cur, con_last);
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    in_contact[f] = con_cur[f] > 0.f;
    feetF[f] = fz_sum[f] / (float)ZB_V4_HIST;  // mean over the history (v4.py:846-849)
  }
  const float ep_len = CST(ZB_V4_EP_LEN) + 1.f;
  float cmd[2] = {CST(ZB_V4_COMMANDS), CST(ZB_V4_COMMANDS + 1)};
  float tgt = CST(ZB_V4_TARGET_YAW);
  float ileft = CST(ZB_V4_INTERVAL_LEFT);
  float f_last[2] = {CST(ZB_V4_FEET_F_LAST), CST(ZB_V4_FEET_F_LAST + 1)};
  float step_len[2] = {CST(ZB_V4_FEET_STEP_LEN), CST(ZB_V4_FEET_STEP_LEN + 1)};
  float down[2][3];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int a = 0; a < 3; ++a) down[f][a] = CST(ZB_V4_FEET_DOWN_POS + 3 * f + a);
  float sums0[ZB_V4_NUM_REWARD_TERMS];
#pragma unroll
  for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) sums0[t] = CST(ZB_V4_EP_SUMS + t);
  const int stage = cnt->stage;

  // _compute_intermediate_values (v4.py:809-849) on the post-step state
  float bq[4], sh[3], fwd[3], vb[3], feet[2][3], fzax[2][3], fxax[2][3], fvel[2][3];
  bool died;
  {
    wave_sync();
    fk_team_pose(p, q);
    wave_sync();
    float S[ND][6], org[ND][3];
    read_joints(q, S, org);
    float bp[3], R[9], fq[4];
    link_pose_q(m, q, 6, bp, bq);
    qmat(bq, R);
    sh[0] = R[2]; sh[1] = R[5]; sh[2] = R[8];            // quat_apply(base_quat, z)
    fwd[0] = sh[1]; fwd[1] = -sh[0]; fwd[2] = 0.f;       // GRAVITY_VEC_W x shoulder
    link_origin_vel_q(m, q, p, S, 6, vb);                // body_link_lin_vel_w[base]
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int l = f == 0 ? 0 : 11;
      link_pose_q(m, q, l, feet[f], fq);
#pragma unroll
      for (int a = 0; a < 3; ++a) feet[f][a] += p.pos[a];
      qmat(fq, R);
      const float sg = f == 0 ? 1.f : -1.f;
      fzax[f][0] = sg * R[2]; fzax[f][1] = sg * R[5]; fzax[f][2] = sg * R[8];
      fxax[f][0] = R[0]; fxax[f][1] = R[3]; fxax[f][2] = R[6];
      link_com_vel_q(m, q, p, S, l, fvel[f]);            // body_com_lin_vel_w[feet]
    }
    const float base_z = bp[2] + p.pos[2];
    // _get_dones (v4.py:896-918)
    const float fm = fm_max;
    died = fm > cfg.undesired_force_threshold || base_z < cfg.termination_height;
  }
  const bool time_out = ep_len >= (float)(cfg.max_episode_length - 1);
  const bool blowup = phys_bad(p);  // non-finite guard (phys_bad), as in the walking kernel
  died |= blowup;
  float cur_yaw = atan2f(fwd[1], fwd[0]);
  float he;
  {
    float sn, cs;
    sincos_r(tgt - cur_yaw, &sn, &cs);
    he = atan2f(sn, cs);
  }
  const float vfwd = dot3(vb, fwd);

  // _get_rewards (v4.py:883-894), terms 1003-1171 in dict order
  float r[ZB_V4_NUM_REWARD_TERMS];
  {
    const float e = cmd[0] - vfwd;
    r[ZB_V4_R_TRACK_LIN_VEL_X] = __expf(-e * e / 0.25f);
    r[ZB_V4_R_TRACK_HEADING_YAW] = __expf(-he * he / 0.25f);
    const float vy = dot3(vb, sh);
    r[ZB_V4_R_LIN_VEL_Y] = vy * vy;
    r[ZB_V4_R_ACTION_RATE] = pr.action_rate;
    r[ZB_V4_R_TORQUES] = so.tau2;
    float jv = 0.f, ja = 0.f;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      jv += p.jqd[j] * p.jqd[j];
      const float aj = (p.jqd[j] - pr.jqd_prev[j]) / cfg.sim_dt;
      ja += aj * aj;
    }
    r[ZB_V4_R_JOINT_VEL] = jv;
    r[ZB_V4_R_JOINT_ACC] = ja;
    float sd = 0.f, sfw = 0.f;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const float dz[3] = {fzax[f][0], fzax[f][1], fzax[f][2] - 1.f};
      sd += sqrtf(dot3(dz, dz));
      const float dx[3] = {fxax[f][0] - fwd[0], fxax[f][1] - fwd[1], fxax[f][2] - fwd[2]};
      sfw += sqrtf(dot3(dx, dx));
    }
    r[ZB_V4_R_FEET_DOWNWARD] = sd;
    r[ZB_V4_R_FEET_FORWARD] = sfw;
    // step_length (v4.py:1058-1095): touchdown foot records its step along the heading, signed by
    // the commanded direction; the stored lengths decay by 0.99 per step
    const float csg = cmd[0] > 0.f ? 1.f : (cmd[0] < 0.f ? -1.f : 0.f);
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      if (feetF[f] > 10.f && f_last[f] < 10.f) {
        const float dv[3] = {feet[f][0] - down[f][0], feet[f][1] - down[f][1], feet[f][2] - down[f][2]};
        step_len[f] = dot3(dv, fwd) * csg;
#pragma unroll
        for (int a = 0; a < 3; ++a) down[f][a] = feet[f][a];
      }
    }
    const float mn = fminf(step_len[0], step_len[1]);
    step_len[0] *= 0.99f;
    step_len[1] *= 0.99f;
    f_last[0] = feetF[0];
    f_last[1] = feetF[1];
    r[ZB_V4_R_STEP_LENGTH] = tanh_r(15.f * mn);
    // feet_air_time_biped (1129-1143)
    const bool single = (in_contact[0] ? 1 : 0) + (in_contact[1] ? 1 : 0) == 1;
    float bi = 3.4e38f;
#pragma unroll
    for (int f = 0; f < 2; ++f) bi = fminf(bi, single ? (in_contact[f] ? con_cur[f] : air_cur[f]) : 0.f);
    r[ZB_V4_R_FEET_AIR_TIME_BIPED] = fminf(bi, 2.f);
    // airtime_variance (1097-1103): unbiased variance of two values = (a - b)^2 / 2
    const float da = fminf(air_last[0], 0.5f) - fminf(air_last[1], 0.5f);
    const float dc = fminf(con_last[0], 0.5f) - fminf(con_last[1], 0.5f);
    r[ZB_V4_R_AIRTIME_VARIANCE] = 0.5f * da * da + 0.5f * dc * dc;
    float sl = 0.f;
#pragma unroll
    for (int f = 0; f < 2; ++f)
      sl += sqrtf(fvel[f][0] * fvel[f][0] + fvel[f][1] * fvel[f][1]) * (feetF[f] > 1.f ? 1.f : 0.f);
    r[ZB_V4_R_FEET_SLIDE] = sl;
    r[ZB_V4_R_FEET_HARMONY] = (air_last[0] + air_last[1]) - 3.f * fabsf(air_last[0] - air_last[1]);
    const float dx = feet[0][0] - feet[1][0], dy = feet[0][1] - feet[1][1];
    r[ZB_V4_R_FEET_CLOSE] = fmaxf(0.115f - sqrtf(dx * dx + dy * dy), 0.f);
  }
  float reward = 0.f, sums[ZB_V4_NUM_REWARD_TERMS];
#pragma unroll
  for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) {
    const float v = (r[t] * stage_weight(cfg, stage, t)) * step_dt;
    reward += v;
    sums[t] = sums0[t] + v;
  }
  if (died) reward -= cfg.terminal_penalty;  // v4.py:892-893
  if (blowup) {  // finite reward, the episode sums without this step
    reward = -cfg.terminal_penalty;
#pragma unroll
    for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) sums[t] = sums0[t];
  }
  const bool reset = died || time_out;
  const uint64_t hs = env_hash(seed, cnt->calls, i);
  float obs_q[4] = {bq[0], bq[1], bq[2], bq[3]};

  // _reset_idx (v4.py:920-1001): log (sum / own duration), reset events (pose, commands), defaults
  const uint64_t lmask = __ballot(reset && lead);
  if (reset) {
    if (lead) {
      const float dur = fmaxf(ep_len * step_dt, step_dt);
      float* lr = log_row(q);
#pragma unroll
      for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) lr[t] = sums[t] / dur;
      lr[ACC_NRES] = 1.f;
      lr[ACC_DIED] = died ? 1.f : 0.f;
      lr[ACC_TOUT] = time_out ? 1.f : 0.f;
    }
    cur_yaw = reset_pose(m, cfg, hs, p);
    v4_resample(cfg, cnt, hs, 5, cur_yaw, cmd, tgt);
    const float4 qr = q.dflt()[3];
    const float qrel[4] = {qr.x, qr.y, qr.z, qr.w};
    qmul(p.quat, qrel, obs_q);
    float R[9];
    qmat(p.quat, R);
#pragma unroll
    for (int f = 0; f < 2; ++f) {  // feet_down_pos_last: pre-reset feet (v4.py:996) or reset pose's
      const float4 fr = q.dflt()[4 + f];
      const float v[3] = {fr.x, fr.y, fr.z};
      float w3[3];
      mv3(R, v, w3);
#pragma unroll
      for (int a = 0; a < 3; ++a) down[f][a] = (cfg.reset_feet_refresh || blowup) ? p.pos[a] + w3[a] : feet[f][a];
      f_last[f] = cfg.feet_f_last_init;
      step_len[f] = 0.f;
    }
  }
  // interval_command_resample (mode "interval", 3-6 s per env; after the resets, v4.py:426-439)
  ileft -= step_dt;
  if (ileft < 1e-6f) {
    ileft = draw(hs, 8) * (cfg.cmd_interval_s[1] - cfg.cmd_interval_s[0]) + cfg.cmd_interval_s[0];
    v4_resample(cfg, cnt, hs, 9, cur_yaw, cmd, tgt);
  }
  float he_obs;
  {
    float sn, cs;
    sincos_r(tgt - cur_yaw, &sn, &cs);
    he_obs = atan2f(sn, cs);
  }
  log_flush(q, lmask, acc);
  {
    // (an opaque 32-bit index: the load's address is not kept across the physics in a 64-bit register)
    unsigned wi = (unsigned)(q.s * N + i);
    asm volatile("" : "+v"(wi));
    wc[wi] = reset ? wc_invalid(q.s) : wc_row;
  }
  sp.mark(12);
#define OUT(f) q.stg(f)
  if (writer) {
    auto live = [reset](float v) { return reset ? 0.f : v; };
#pragma unroll
    for (int a = 0; a < 3; ++a) { OUT(ZB_S_ROOT_POS + a) = p.pos[a]; OUT(ZB_S_ROOT_LINVEL + a) = p.lv[a]; OUT(ZB_S_ROOT_ANGVEL + a) = p.av[a]; }
#pragma unroll
    for (int a = 0; a < 4; ++a) OUT(ZB_S_ROOT_QUAT + a) = p.quat[a];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      OUT(ZB_S_JOINT_POS + j) = p.jq[j]; OUT(ZB_S_JOINT_VEL + j) = p.jqd[j];
      OUT(ZB_V4_P_DELTA + j) = live(pr.pdel[j]); OUT(ZB_V4_ACTIONS + j) = live(pr.a_now[j]);
    }
    OUT(ZB_V4_COMMANDS) = cmd[0];
    OUT(ZB_V4_COMMANDS + 1) = cmd[1];
    OUT(ZB_V4_TARGET_YAW) = tgt;
    OUT(ZB_V4_INTERVAL_LEFT) = ileft;
    OUT(ZB_V4_CURRENT_YAW) = cur_yaw;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
#pragma unroll
      for (int a = 0; a < 3; ++a) OUT(ZB_V4_FEET_DOWN_POS + 3 * f + a) = down[f][a];
      OUT(ZB_V4_FEET_STEP_LEN + f) = step_len[f];
      OUT(ZB_V4_FEET_F_LAST + f) = f_last[f];
      OUT(ZB_V4_FEET_AIR_CUR + f) = live(air_cur[f]);
      OUT(ZB_V4_FEET_CONTACT_CUR + f) = live(con_cur[f]);
      OUT(ZB_V4_FEET_AIR_LAST + f) = live(air_last[f]);
      OUT(ZB_V4_FEET_CONTACT_LAST + f) = live(con_last[f]);

    }
    sens_store<ZB_V4_HIST>(q, cst, 1, 0, ZB_V4_FEET_FZ_HIST, ZB_V4_UNDES_FMAX_HIST, cfg.decimation, reset,
                           [&](int row, float v) { OUT(row) = v; });
    OUT(ZB_V4_EP_LEN) = live(ep_len);
#pragma unroll
    for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) OUT(ZB_V4_EP_SUMS + t) = live(sums[t]);

    // _get_observations (v4.py:851-881)
    float* o = &q.stg(ZB_V4_STATE_DIM);
    o[0] = obs_q[0]; o[1] = obs_q[1]; o[2] = obs_q[2]; o[3] = obs_q[3];
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      o[4 + j] = p.jq[j] - m->default_joint_pos[j];
      o[10 + j] = p.jqd[j];
      o[16 + j] = live(pr.a_now[j]);
    }
    o[22] = cmd[0];
    o[23] = he_obs;
    q.stg(ZB_V4_STATE_DIM + ZB_V4_OBS_DIM) = reward;
    q.stg(ZB_V4_STATE_DIM + ZB_V4_OBS_DIM + 1) = died ? 1.f : 0.f;
    q.stg(ZB_V4_STATE_DIM + ZB_V4_OBS_DIM + 2) = time_out ? 1.f : 0.f;
  }
  staged_store<ZB_V4_STATE_DIM, ZB_V4_OBS_DIM>(q, xcd_block(blockIdx.x, gridDim.x) * EPW, N, st, obs, rew, term, trunc, done);
#undef OUT
  sp.mark(8);
  sp.flush();
#undef ST
#undef CST
}

// explicit resets / construction (init = 1 also draws the interval-event timers, as Isaac Lab's
// EventManager does when it is created): log, reset events, defaults; one thread per env
__global__ void zb_v4_reset_kernel(const zb_model* __restrict__ mg, const float4* __restrict__ links, zb_task_cfg cfg,
                                   int N, float* __restrict__ st, const int32_t* __restrict__ ids, int n,
                                   float* __restrict__ acc, const Counters* __restrict__ cnt, uint64_t seed, int init) {
  MP m = to_mp(mg);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int i = ids ? ids[t] : t;
  if (i < 0 || i >= N) return;
#define ST(f) st[(size_t)(f) * N + i]
  const float step_dt = cfg.sim_dt * (float)cfg.decimation;
  if (!init) {
    const float dur = fmaxf(ST(ZB_V4_EP_LEN) * step_dt, step_dt);
#pragma unroll
    for (int k = 0; k < ZB_V4_NUM_REWARD_TERMS; ++k) atomicAdd(&acc_slot(acc, t)[k], ST(ZB_V4_EP_SUMS + k) / dur);
    atomicAdd(&acc_slot(acc, t)[ACC_NRES], 1.f);
  }
  float pre[2][3];  // the pre-reset feet (the spawn pose at construction)
  if (!cfg.reset_feet_refresh) {
    Phys p0;
    if (init) phys_default(m, p0);
    else load_phys(st, N, i, p0);
    feet_world(m, p0, pre);
  }
  Phys p;
  const uint64_t hs = env_hash(seed, cnt->calls, i);
  const float cur_yaw = reset_pose(m, cfg, hs, p);
  float cmd[2], tgt;
  v4_resample(cfg, cnt, hs, 5, cur_yaw, cmd, tgt);
#pragma unroll
  for (int a = 0; a < 3; ++a) { ST(ZB_S_ROOT_POS + a) = p.pos[a]; ST(ZB_S_ROOT_LINVEL + a) = p.lv[a]; ST(ZB_S_ROOT_ANGVEL + a) = p.av[a]; }
#pragma unroll
  for (int a = 0; a < 4; ++a) ST(ZB_S_ROOT_QUAT + a) = p.quat[a];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    ST(ZB_S_JOINT_POS + j) = p.jq[j]; ST(ZB_S_JOINT_VEL + j) = p.jqd[j];
    ST(ZB_V4_P_DELTA + j) = 0.f; ST(ZB_V4_ACTIONS + j) = 0.f;
  }
  ST(ZB_V4_COMMANDS) = cmd[0];
  ST(ZB_V4_COMMANDS + 1) = cmd[1];
  ST(ZB_V4_TARGET_YAW) = tgt;
  ST(ZB_V4_CURRENT_YAW) = cur_yaw;
  if (init) ST(ZB_V4_INTERVAL_LEFT) = draw(hs, 8) * (cfg.cmd_interval_s[1] - cfg.cmd_interval_s[0]) + cfg.cmd_interval_s[0];
  float R[9];
  qmat(p.quat, R);
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const float4 fr = links[DFLT_OFF + 4 + f];
    const float v[3] = {fr.x, fr.y, fr.z};
    float w3[3];
    mv3(R, v, w3);
#pragma unroll
    for (int a = 0; a < 3; ++a) ST(ZB_V4_FEET_DOWN_POS + 3 * f + a) = cfg.reset_feet_refresh ? p.pos[a] + w3[a] : pre[f][a];
    ST(ZB_V4_FEET_STEP_LEN + f) = 0.f;
    ST(ZB_V4_FEET_F_LAST + f) = cfg.feet_f_last_init;
    ST(ZB_V4_FEET_AIR_CUR + f) = 0.f;
    ST(ZB_V4_FEET_CONTACT_CUR + f) = 0.f;
    ST(ZB_V4_FEET_AIR_LAST + f) = 0.f;
    ST(ZB_V4_FEET_CONTACT_LAST + f) = 0.f;
#pragma unroll
    for (int h = 0; h < ZB_V4_HIST; ++h) ST(ZB_V4_FEET_FZ_HIST + 2 * h + f) = 0.f;
  }
#pragma unroll
  for (int h = 0; h < ZB_V4_HIST; ++h) ST(ZB_V4_UNDES_FMAX_HIST + h) = 0.f;
  ST(ZB_V4_EP_LEN) = 0.f;
#pragma unroll
  for (int k = 0; k < ZB_V4_NUM_REWARD_TERMS; ++k) ST(ZB_V4_EP_SUMS + k) = 0.f;
#undef ST
}

__global__ void zb_v4_observe_kernel(const zb_model* __restrict__ mg, int N, const float* __restrict__ st,
                                     float* __restrict__ obs) {
  MP m = to_mp(mg);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  Phys p;
  load_phys(st, N, i, p);
  Kin k;
  fk(m, p, k);
  float bp[3], bq[4];
  link_pose(m, k, 6, bp, bq);
  float* o = obs + (size_t)i * ZB_V4_OBS_DIM;
  o[0] = bq[0]; o[1] = bq[1]; o[2] = bq[2]; o[3] = bq[3];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    o[4 + j] = p.jq[j] - m->default_joint_pos[j];
    o[10 + j] = p.jqd[j];
    o[16 + j] = st[(size_t)(ZB_V4_ACTIONS + j) * N + i];
  }
  o[22] = st[(size_t)ZB_V4_COMMANDS * N + i];
  float sn, cs;
  sincos_r(st[(size_t)ZB_V4_TARGET_YAW * N + i] - st[(size_t)ZB_V4_CURRENT_YAW * N + i], &sn, &cs);
  o[23] = atan2f(sn, cs);
}

// =========================================================================== manager-based env
// zbot-6b-walking-m-v0 (reference tasks/zbotlab_manager: zbotlab_env_cfg.py = "mgr.py",
// config/zbot6b_manager/flat_env_cfg.py, mdp/rewards.py, terminations.py, curriculums.py) on
// ZBOT_6S_V2_CFG (zbot_6s_v09.usd, rooted at the base link). ManagerBasedRLEnv.step order: action
// (RelativeJointPositionAction re-targets q + delta every substep), 4 x (substep, scene.update:
// the contact sensor with history_length 3 > 0 updates every physics step), terminations,
// rewards, resets (curriculum, events, managers), command update, observations with noise.

// world angular velocity of body b (root twist + the joint rates before it)
__device__ __forceinline__ void body_ang_vel_q(const Phys& s, const float S[ND][6], int b, float w[3]) {
  w[0] = s.av[0]; w[1] = s.av[1]; w[2] = s.av[2];
#pragma unroll
  for (int j = 0; j < ND; ++j)
    if (j < b)
#pragma unroll
      for (int a = 0; a < 3; ++a) w[a] += S[j][a] * s.jqd[j];
}

// UniformVelocityCommand._resample_command: lin x ~ U(ranges.lin_vel_x) (cnt->vel), lin y ~
// U(ranges.lin_vel_y) (cnt->yaw holds the lin_vel_y range for this task), ang z ~ U(0, 0),
// standing ~ U(0, 1) <= rel_standing_envs; draws k0 .. k0 + 2
__device__ __forceinline__ void m_resample(const zb_task_cfg& cfg, const Counters* cnt, uint64_t h, int k0, float cmd[3],
                                           float& standing) {
  cmd[0] = draw(h, k0) * (cnt->vel[1] - cnt->vel[0]) + cnt->vel[0];
  cmd[1] = draw(h, k0 + 1) * (cnt->yaw[1] - cnt->yaw[0]) + cnt->yaw[0];
  cmd[2] = 0.f;
  standing = draw(h, k0 + 2) <= cfg.cmd_rel_standing ? 1.f : 0.f;
}
constexpr int M_DRAW_RESET_CMD = 5, M_DRAW_CMD = 9, M_DRAW_NOISE = 16;  // reset_pose uses draws 1..4

// the policy observation group (mgr.py:136-161, corruption on): root quat, command, joint pos rel,
// joint vel rel (Isaac Lab joint order), last action; additive U(-n, n) noise from draws 16..37
__device__ __forceinline__ void m_write_obs(MP m, const zb_task_cfg& cfg, uint64_t h, const float bq[4],
                                            const float cmd[3], const Phys& p, const float a_obs[ND], float* o) {
  const float cor = cfg.obs_corruption ? 1.f : 0.f;
  auto noise = [&](int k, float n) { return cor * (draw(h, M_DRAW_NOISE + k) * (2.f * n) - n); };
#pragma unroll
  for (int a = 0; a < 4; ++a) o[a] = bq[a] + noise(a, cfg.obs_noise[0]);
#pragma unroll
  for (int a = 0; a < 3; ++a) o[4 + a] = cmd[a];
#pragma unroll
  for (int j = 0; j < ND; ++j) {
    const int ai = m->api_joint_index[j];
    const float sg = m->api_joint_sign[j];
    o[7 + ai] = sg * (p.jq[j] - m->default_joint_pos[j]) + noise(4 + ai, cfg.obs_noise[1]);
    o[13 + ai] = sg * p.jqd[j] + noise(10 + ai, cfg.obs_noise[2]);
  }
#pragma unroll
  for (int a = 0; a < ND; ++a) o[19 + a] = a_obs[a];
}

struct PreM {
  float delta[ND], jqd_prev[ND], a_raw[ND], action_rate;
};
static_assert(sizeof(PreM) <= 16 * PRE4, "PreM fits PRE4 granules");

template <bool kTgs, int kOcc>
__global__ __launch_bounds__(WGT, kOcc) void zb_m_step_kernel(
    const zb_model* __restrict__ mg, const float4* __restrict__ links, zb_task_cfg cfg, int N, float* __restrict__ st,
    const float* __restrict__ act, float* __restrict__ obs, float* __restrict__ rew, uint8_t* __restrict__ term,
    uint8_t* __restrict__ trunc, int64_t* __restrict__ done, float* __restrict__ acc,
    const Counters* __restrict__ cnt, uint64_t seed, float* __restrict__ wc) {
  MP m = to_mp(mg);
  __shared__ float4 lds[LDS4];
  if (kOcc == 1) asm volatile("" ::: "a255");  // (zb_step_kernel: kOcc)
  const int lane = threadIdx.x;
  const int env = xcd_block(blockIdx.x, gridDim.x) * EPW + lane / TL;
  const int i = env < N ? env : N - 1;
  const bool lead = env < N && lane % TL == 0;
  const Q q = make_q(lds, lane, links);
  for (int t = LNK_G + lane; t < LNK4; t += WGT) lds[LNK_OFF + t] = links[t];
  Stamps sp;
  sp.begin();
#define ST(f) st[(size_t)(f) * N + i]
  Phys p;
#pragma unroll
  for (int a = 0; a < 3; ++a) { p.pos[a] = ST(ZB_S_ROOT_POS + a); p.lv[a] = ST(ZB_S_ROOT_LINVEL + a); p.av[a] = ST(ZB_S_ROOT_ANGVEL + a); }
#pragma unroll
  for (int a = 0; a < 4; ++a) p.quat[a] = ST(ZB_S_ROOT_QUAT + a);
#pragma unroll
  for (int j = 0; j < ND; ++j) { p.jq[j] = ST(ZB_S_JOINT_POS + j); p.jqd[j] = ST(ZB_S_JOINT_VEL + j); }
  const float* cst = carry_prefetch<ZB_M_LINK_MU>(q, st, N, i);  // the friction rows load into FRIC
#define CST(f) cst[f]
  if (q.s < NL) {
    q.fric(q.s) = ST(ZB_M_LINK_MU + q.s);
    q.fricd(q.s) = ST(ZB_M_LINK_MU_D + q.s);
  }

  // ActionManager.process_action: RelativeJointPositionAction (scale 0.04 pi, zero offset, clip
  // +-0.04 pi) in the Isaac Lab joint order, mapped onto the chain's joints
  const bool writer = q.s == 0;
  const float step_dt = cfg.sim_dt * (float)cfg.decimation;
  PreM& pv = *reinterpret_cast<PreM*>(&q.pre());
  float delta[ND];
  {
    PreM pr;
    pr.action_rate = 0.f;
#pragma unroll
    for (int a = 0; a < ND; ++a) {
      pr.a_raw[a] = act[(size_t)i * ZB_ACT_DIM + a];
      const float d = pr.a_raw[a] - ST(ZB_M_ACTIONS + a);
      pr.action_rate += d * d;
    }
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      float a = pr.a_raw[0];
#pragma unroll
      for (int b = 1; b < ND; ++b) a = m->api_joint_index[j] == b ? pr.a_raw[b] : a;
      delta[j] = m->api_joint_sign[j] * clampf(a * cfg.action_scale, -cfg.action_clip, cfg.action_clip);
      pr.jqd_prev[j] = 0.f;
    }
    if (writer) pv = pr;
  }

  // 4 x (apply_action: target = q + delta from the current joint positions; physics step;
  // ContactSensor.update: feet net force into the 3-slot history, air-time timers + sim_dt).
  // With 4 substeps the 3 history slots are this step's substeps 2..4.
  SensorOut so;
  float fz_h[3][2], fn_h[3][2];
  float air_cur[2] = {ST(ZB_M_FEET_AIR_CUR), ST(ZB_M_FEET_AIR_CUR + 1)};
  float air_last[2] = {ST(ZB_M_FEET_AIR_LAST), ST(ZB_M_FEET_AIR_LAST + 1)};
  const bool hist_in = cfg.decimation < 3;  // >= 3 substeps overwrite every slot: no read
#pragma unroll
  for (int h = 0; h < 3; ++h)
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      fz_h[h][f] = hist_in ? ST(ZB_M_FEET_FZ_HIST + 2 * h + f) : 0.f;
      fn_h[h][f] = hist_in ? ST(ZB_M_FEET_FN_HIST + 2 * h + f) : 0.f;
    }
  wc_load(q, wc, N, i);  // the first substep's GJK warm start
  sp.mark(0);
  for (int k = 0; k < cfg.decimation; ++k) {
    float target[ND];
#pragma unroll
    for (int j = 0; j < ND; ++j) target[j] = p.jq[j] + delta[j];
    if (k == cfg.decimation - 1 && writer) {
#pragma unroll
      for (int j = 0; j < ND; ++j) pv.jqd_prev[j] = p.jqd[j];
    }
    substep<false, true, kTgs>(m, cfg, p, target, q, true, true, so, nullptr, nullptr, sp);
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const float fn = sqrtf(dot3(so.feet_f[f], so.feet_f[f]));
      fz_h[2][f] = fz_h[1][f]; fz_h[1][f] = fz_h[0][f]; fz_h[0][f] = so.feet_f[f][2];
      fn_h[2][f] = fn_h[1][f]; fn_h[1][f] = fn_h[0][f]; fn_h[0][f] = fn;
      const bool c = fn > cfg.contact_force_threshold;
      air_last[f] = (air_cur[f] > 0.f && c) ? air_cur[f] + cfg.sim_dt : air_last[f];
      air_cur[f] = c ? 0.f : air_cur[f] + cfg.sim_dt;
    }
    sp.mark(7);
  }
  m = opaque(m);
  wave_sync();
  const float wc_row = wc_extract(q);
  const PreM pr = pv;
  st = opaque_ptr(st);

  const float ep_len = CST(ZB_M_EP_LEN) + 1.f;
  float cmd[3] = {CST(ZB_M_COMMANDS), CST(ZB_M_COMMANDS + 1), CST(ZB_M_COMMANDS + 2)};
  float tleft = CST(ZB_M_CMD_TIME_LEFT), standing = CST(ZB_M_CMD_STANDING);
  float met[2] = {CST(ZB_M_METRICS), CST(ZB_M_METRICS + 1)};
  float f_last[2] = {CST(ZB_M_FEET_F_LAST), CST(ZB_M_FEET_F_LAST + 1)};
  float step_len[2] = {CST(ZB_M_FEET_STEP_LEN), CST(ZB_M_FEET_STEP_LEN + 1)};
  float down[2][3];
#pragma unroll
  for (int f = 0; f < 2; ++f)
#pragma unroll
    for (int a = 0; a < 3; ++a) down[f][a] = CST(ZB_M_FEET_DOWN_POS + 3 * f + a);

  // post-step articulation data: root (= base link) pose, link-origin / COM velocity, angular
  // velocity; feet link poses and COM velocities
  float bq[4], bp[3], vb[3], vcom[3], wb[3], feet[2][3], fq[2][4], fvel[2][3];
  {
    wave_sync();
    fk_team_pose(p, q);
    wave_sync();
    float S[ND][6], org[ND][3];
    read_joints(q, S, org);
    const int B = m->base_link;
    link_pose_q(m, q, B, bp, bq);
#pragma unroll
    for (int a = 0; a < 3; ++a) bp[a] += p.pos[a];
    link_origin_vel_q(m, q, p, S, B, vb);
    link_com_vel_q(m, q, p, S, B, vcom);
    body_ang_vel_q(p, S, link_body(B), wb);
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const int l = f == 0 ? 0 : 11;
      link_pose_q(m, q, l, feet[f], fq[f]);
#pragma unroll
      for (int a = 0; a < 3; ++a) feet[f][a] += p.pos[a];
      link_com_vel_q(m, q, p, S, l, fvel[f]);
    }
  }
  // TerminationManager (flat: time_out, base_height < 0.2, feet_close < 0.12)
  const bool time_out = ep_len >= (float)cfg.max_episode_length;
  const bool low = bp[2] < cfg.termination_height;
  const float fd[3] = {feet[0][0] - feet[1][0], feet[0][1] - feet[1][1], feet[0][2] - feet[1][2]};
  const bool close = sqrtf(dot3(fd, fd)) < cfg.feet_close_min;
  const bool blowup = phys_bad(p);  // non-finite guard (phys_bad), as in the walking kernel
  const bool terminated = low || close || blowup;

  // RewardManager.compute: term * weight * step_dt in cfg order (mgr.py:262-357, flat overrides)
  float r[ZB_M_NUM_REWARD_TERMS];
  {
    float Rb[9];
    qmat(bq, Rb);
    const float fwd[3] = {Rb[4], -Rb[1], 0.f};  // GRAVITY_VEC_W x quat_apply(root_quat, y)
    float vx, vy;
    {  // yaw_quat + quat_apply_inverse on root_link_lin_vel_w
      const float yaw = atan2f(2.f * (bq[0] * bq[3] + bq[1] * bq[2]), 1.f - 2.f * (bq[2] * bq[2] + bq[3] * bq[3]));
      float sy, cy;
      sincos_r(yaw, &sy, &cy);
      vx = cy * vb[0] + sy * vb[1];
      vy = -sy * vb[0] + cy * vb[1];
    }
    const float ex = cmd[0] - vx, ey = cmd[1] - vy;
    r[ZB_M_R_TRACK_LIN_VEL_XY] = __expf(-(ex * ex + ey * ey) / 0.25f);
    const float ez = cmd[2] - wb[2];
    r[ZB_M_R_TRACK_ANG_VEL_Z] = __expf(-(ez * ez) / 0.25f);
    r[ZB_M_R_TERMINATION] = terminated ? 1.f : 0.f;
    r[ZB_M_R_DOF_TORQUES] = so.tau2;
    float ja = 0.f;
#pragma unroll
    for (int j = 0; j < ND; ++j) {
      const float aj = (p.jqd[j] - pr.jqd_prev[j]) / cfg.sim_dt;
      ja += aj * aj;
    }
    r[ZB_M_R_DOF_ACC] = ja;
    r[ZB_M_R_ACTION_RATE] = pr.action_rate;
    // foot_step_length (rewards.py:44-104)
    const float nrm = sqrtf(dot3(fwd, fwd)) + 1e-6f;
    const float fh[3] = {fwd[0] / nrm, fwd[1] / nrm, fwd[2] / nrm};
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      const float fz = (fz_h[0][f] + fz_h[1][f] + fz_h[2][f]) / 3.f;
      if (fz > 10.f && f_last[f] < 10.f) {
        const float dv[3] = {feet[f][0] - down[f][0], feet[f][1] - down[f][1], feet[f][2] - down[f][2]};
        step_len[f] = fabsf(dot3(dv, fh));
#pragma unroll
        for (int a = 0; a < 3; ++a) down[f][a] = feet[f][a];
      }
      f_last[f] = fz;
    }
    r[ZB_M_R_FOOT_STEP_LENGTH] = tanh_r(15.f * fminf(step_len[0], step_len[1]));
    float sd = 0.f, sfw = 0.f, sl = 0.f;
#pragma unroll
    for (int f = 0; f < 2; ++f) {
      float R[9];
      qmat(fq[f], R);
      const float sg = f == 0 ? 1.f : -1.f;  // foot_downward: feet axes (0, 1, 0), (0, -1, 0) vs z
      const float dz[3] = {sg * R[1], sg * R[4], sg * R[7] - 1.f};
      sd += sqrtf(dot3(dz, dz));
      const float dx[3] = {R[0] - fwd[0], R[3] - fwd[1], R[6] - fwd[2]};  // foot_forward
      sfw += sqrtf(dot3(dx, dx));
      const bool c = fmaxf(fn_h[0][f], fmaxf(fn_h[1][f], fn_h[2][f])) > 1.0f;  // feet_slide
      sl += sqrtf(fvel[f][0] * fvel[f][0] + fvel[f][1] * fvel[f][1]) * (c ? 1.f : 0.f);
    }
    r[ZB_M_R_FOOT_DOWNWARD] = sd;
    r[ZB_M_R_FOOT_FORWARD] = sfw;
    r[ZB_M_R_FEET_SLIDE] = sl;
    r[ZB_M_R_AIR_TIME_BALANCE] = fabsf(air_last[0] - air_last[1]);
  }
  float reward = 0.f, sums[ZB_M_NUM_REWARD_TERMS];
#pragma unroll
  for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) {
    const float v = r[t] * cfg.stage_scales[0][t] * step_dt;
    reward += v;
    sums[t] = CST(ZB_M_EP_SUMS + t) + v;
  }
  if (blowup) {  // finite reward (the is_terminated term alone), the episode sums without this step
    reward = cfg.stage_scales[0][ZB_M_R_TERMINATION] * step_dt;
#pragma unroll
    for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) sums[t] = CST(ZB_M_EP_SUMS + t);
  }
  const bool reset = terminated || time_out;
  const uint64_t hs = env_hash(seed, cnt->calls, i);
  float a_obs[ND];
#pragma unroll
  for (int a = 0; a < ND; ++a) a_obs[a] = pr.a_raw[a];
  float vcb[3], wcb[3];  // root_lin_vel_b (COM), root_ang_vel_b after the resets

  // _reset_idx: curriculum (finalize), events reset_base / reset_robot_joints / reset_my_data,
  // managers (actions 0, reward sums and metrics logged, command resampled, sensor cleared)
  const uint64_t lmask = __ballot(reset && lead);
  if (reset) {
    if (lead) {
      float* lr = log_row(q);
#pragma unroll
      for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) lr[t] = sums[t];
      lr[ACC_NRES] = 1.f;
      lr[ACC_DIED] = low ? 1.f : 0.f;
      lr[ACC_TOUT] = time_out ? 1.f : 0.f;
      lr[ACC_TERM2] = close ? 1.f : 0.f;
      lr[ACC_MET0] = met[0];
      lr[ACC_MET1] = met[1];
    }
    (void)reset_pose(m, cfg, hs, p);
    const float4 qr = q.dflt()[3];
    const float qrel[4] = {qr.x, qr.y, qr.z, qr.w};
    qmul(p.quat, qrel, bq);
    float R[9];
    qmat(p.quat, R);
#pragma unroll
    for (int f = 0; f < 2; ++f) {  // reset_my_data: pre-reset feet (rewards.py:42) or reset pose's
      const float4 fr = q.dflt()[4 + f];
      const float v[3] = {fr.x, fr.y, fr.z};
      float w3[3];
      mv3(R, v, w3);
#pragma unroll
      for (int a = 0; a < 3; ++a) down[f][a] = (cfg.reset_feet_refresh || blowup) ? p.pos[a] + w3[a] : feet[f][a];
      f_last[f] = 0.f;
      step_len[f] = 0.f;
    }
    m_resample(cfg, cnt, hs, M_DRAW_RESET_CMD, cmd, standing);
    tleft = cfg.cmd_resample_s;
    met[0] = met[1] = 0.f;
#pragma unroll
    for (int a = 0; a < ND; ++a) a_obs[a] = 0.f;
#pragma unroll
    for (int a = 0; a < 3; ++a) { vcb[a] = 0.f; wcb[a] = 0.f; }
  } else {
    float R[9];
    qmat(bq, R);
    vcb[0] = R[0] * vcom[0] + R[3] * vcom[1] + R[6] * vcom[2];
    vcb[1] = R[1] * vcom[0] + R[4] * vcom[1] + R[7] * vcom[2];
    vcb[2] = R[2] * vcom[0] + R[5] * vcom[1] + R[8] * vcom[2];
    wcb[0] = R[0] * wb[0] + R[3] * wb[1] + R[6] * wb[2];
    wcb[1] = R[1] * wb[0] + R[4] * wb[1] + R[7] * wb[2];
    wcb[2] = R[2] * wb[0] + R[5] * wb[1] + R[8] * wb[2];
  }
  // CommandManager.compute: metrics (UniformVelocityCommand._update_metrics), timer, resample,
  // standing envs zeroed
  {
    const float max_steps = cfg.cmd_resample_s / step_dt;
    const float ex = cmd[0] - vcb[0], ey = cmd[1] - vcb[1];
    met[0] += sqrtf(ex * ex + ey * ey) / max_steps;
    met[1] += fabsf(cmd[2] - wcb[2]) / max_steps;
    tleft -= step_dt;
    if (tleft <= 0.f) {
      m_resample(cfg, cnt, hs, M_DRAW_CMD, cmd, standing);
      tleft = cfg.cmd_resample_s;
    }
    if (standing > 0.5f) cmd[0] = cmd[1] = cmd[2] = 0.f;
  }
  log_flush(q, lmask, acc);
  {
    // (an opaque 32-bit index: the load's address is not kept across the physics in a 64-bit register)
    unsigned wi = (unsigned)(q.s * N + i);
    asm volatile("" : "+v"(wi));
    wc[wi] = reset ? wc_invalid(q.s) : wc_row;
  }
  sp.mark(12);
#define OUT(f) q.stg(f)
  if (writer) {
    auto live = [reset](float v) { return reset ? 0.f : v; };
#pragma unroll
    for (int a = 0; a < 3; ++a) { OUT(ZB_S_ROOT_POS + a) = p.pos[a]; OUT(ZB_S_ROOT_LINVEL + a) = p.lv[a]; OUT(ZB_S_ROOT_ANGVEL + a) = p.av[a]; }
#pragma unroll
    for (int a = 0; a < 4; ++a) OUT(ZB_S_ROOT_QUAT + a) = p.quat[a];
#pragma unroll
    for (int j = 0; j < ND; ++j) { OUT(ZB_S_JOINT_POS + j) = p.jq[j]; OUT(ZB_S_JOINT_VEL + j) = p.jqd[j]; }
#pragma unroll
    for (int a = 0; a < ND; ++a) OUT(ZB_M_ACTIONS + a) = a_obs[a];
#pragma unroll
    for (int a = 0; a < 3; ++a) OUT(ZB_M_COMMANDS + a) = cmd[a];
    OUT(ZB_M_CMD_TIME_LEFT) = tleft;
    OUT(ZB_M_CMD_STANDING) = standing;
    OUT(ZB_M_METRICS) = met[0];
    OUT(ZB_M_METRICS + 1) = met[1];
#pragma unroll
    for (int f = 0; f < 2; ++f) {
#pragma unroll
      for (int a = 0; a < 3; ++a) OUT(ZB_M_FEET_DOWN_POS + 3 * f + a) = down[f][a];
      OUT(ZB_M_FEET_STEP_LEN + f) = step_len[f];
      OUT(ZB_M_FEET_F_LAST + f) = f_last[f];
      OUT(ZB_M_FEET_AIR_CUR + f) = live(air_cur[f]);
      OUT(ZB_M_FEET_AIR_LAST + f) = live(air_last[f]);
#pragma unroll
      for (int h = 0; h < 3; ++h) { OUT(ZB_M_FEET_FZ_HIST + 2 * h + f) = live(fz_h[h][f]); OUT(ZB_M_FEET_FN_HIST + 2 * h + f) = live(fn_h[h][f]); }
    }
    OUT(ZB_M_EP_LEN) = live(ep_len);
#pragma unroll
    for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) OUT(ZB_M_EP_SUMS + t) = live(sums[t]);
    m_write_obs(m, cfg, hs, bq, cmd, p, a_obs, &q.stg(ZB_M_LINK_MU));
    q.stg(ZB_M_LINK_MU + ZB_M_OBS_DIM) = reward;
    q.stg(ZB_M_LINK_MU + ZB_M_OBS_DIM + 1) = terminated ? 1.f : 0.f;
    q.stg(ZB_M_LINK_MU + ZB_M_OBS_DIM + 2) = time_out ? 1.f : 0.f;
  }
  staged_store<ZB_M_LINK_MU, ZB_M_OBS_DIM>(q, xcd_block(blockIdx.x, gridDim.x) * EPW, N, st, obs, rew, term, trunc, done);
#undef OUT
  sp.mark(8);
  sp.flush();
#undef ST
#undef CST
}

// command of a reset env redrawn after lin_vel_cmd_levels widened the ranges (zb_finalize_kernel):
// the post-reset state has zero velocity, so the first metric update reads |command| only
__device__ __forceinline__ void m_fixup_env(const zb_task_cfg& cfg, int N, float* __restrict__ st, float* __restrict__ obs,
                                            const Counters* cnt, uint64_t hs, int i) {
  float cmd[3], standing;
  m_resample(cfg, cnt, hs, M_DRAW_RESET_CMD, cmd, standing);
  const float step_dt = cfg.sim_dt * (float)cfg.decimation;
  const float max_steps = cfg.cmd_resample_s / step_dt;
  const float ex = cmd[0] - 0.f, ey = cmd[1] - 0.f;
  st[(size_t)ZB_M_METRICS * N + i] = 0.f + sqrtf(ex * ex + ey * ey) / max_steps;
  st[(size_t)(ZB_M_METRICS + 1) * N + i] = 0.f + fabsf(cmd[2] - 0.f) / max_steps;
  st[(size_t)ZB_M_CMD_STANDING * N + i] = standing;
  if (standing > 0.5f) cmd[0] = cmd[1] = cmd[2] = 0.f;
#pragma unroll
  for (int a = 0; a < 3; ++a) {
    st[(size_t)(ZB_M_COMMANDS + a) * N + i] = cmd[a];
    obs[(size_t)i * ZB_M_OBS_DIM + 4 + a] = cmd[a];
  }
}

// explicit resets / construction (init: also the friction default): one thread per env. The
// command is resampled but not yet zeroed for standing envs (that happens in the next
// CommandManager.compute, i.e. the next step).
__global__ void zb_m_reset_kernel(const zb_model* __restrict__ mg, const float4* __restrict__ links, zb_task_cfg cfg,
                                  int N, float* __restrict__ st, const int32_t* __restrict__ ids, int n,
                                  float* __restrict__ acc, const Counters* __restrict__ cnt, uint64_t seed, int init) {
  MP m = to_mp(mg);
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int i = ids ? ids[t] : t;
  if (i < 0 || i >= N) return;
#define ST(f) st[(size_t)(f) * N + i]
  if (!init) {
#pragma unroll
    for (int k = 0; k < ZB_M_NUM_REWARD_TERMS; ++k) atomicAdd(&acc_slot(acc, t)[k], ST(ZB_M_EP_SUMS + k));
    atomicAdd(&acc_slot(acc, t)[ACC_NRES], 1.f);
    atomicAdd(&acc_slot(acc, t)[ACC_MET0], ST(ZB_M_METRICS));
    atomicAdd(&acc_slot(acc, t)[ACC_MET1], ST(ZB_M_METRICS + 1));
  }
  float pre[2][3];  // the pre-reset feet (the spawn pose at construction)
  if (!cfg.reset_feet_refresh) {
    Phys p0;
    if (init) phys_default(m, p0);
    else load_phys(st, N, i, p0);
    feet_world(m, p0, pre);
  }
  Phys p;
  const uint64_t hs = env_hash(seed, cnt->calls, i);
  (void)reset_pose(m, cfg, hs, p);
  float cmd[3], standing;
  m_resample(cfg, cnt, hs, M_DRAW_RESET_CMD, cmd, standing);
#pragma unroll
  for (int a = 0; a < 3; ++a) { ST(ZB_S_ROOT_POS + a) = p.pos[a]; ST(ZB_S_ROOT_LINVEL + a) = p.lv[a]; ST(ZB_S_ROOT_ANGVEL + a) = p.av[a]; }
#pragma unroll
  for (int a = 0; a < 4; ++a) ST(ZB_S_ROOT_QUAT + a) = p.quat[a];
#pragma unroll
  for (int j = 0; j < ND; ++j) { ST(ZB_S_JOINT_POS + j) = p.jq[j]; ST(ZB_S_JOINT_VEL + j) = p.jqd[j]; ST(ZB_M_ACTIONS + j) = 0.f; }
#pragma unroll
  for (int a = 0; a < 3; ++a) ST(ZB_M_COMMANDS + a) = cmd[a];
  ST(ZB_M_CMD_TIME_LEFT) = cfg.cmd_resample_s;
  ST(ZB_M_CMD_STANDING) = standing;
  ST(ZB_M_METRICS) = 0.f;
  ST(ZB_M_METRICS + 1) = 0.f;
  float R[9];
  qmat(p.quat, R);
#pragma unroll
  for (int f = 0; f < 2; ++f) {
    const float4 fr = links[DFLT_OFF + 4 + f];
    const float v[3] = {fr.x, fr.y, fr.z};
    float w3[3];
    mv3(R, v, w3);
#pragma unroll
    for (int a = 0; a < 3; ++a) ST(ZB_M_FEET_DOWN_POS + 3 * f + a) = cfg.reset_feet_refresh ? p.pos[a] + w3[a] : pre[f][a];
    ST(ZB_M_FEET_STEP_LEN + f) = 0.f;
    ST(ZB_M_FEET_F_LAST + f) = 0.f;
    ST(ZB_M_FEET_AIR_CUR + f) = 0.f;
    ST(ZB_M_FEET_AIR_LAST + f) = 0.f;
#pragma unroll
    for (int h = 0; h < 3; ++h) { ST(ZB_M_FEET_FZ_HIST + 2 * h + f) = 0.f; ST(ZB_M_FEET_FN_HIST + 2 * h + f) = 0.f; }
  }
  ST(ZB_M_EP_LEN) = 0.f;
#pragma unroll
  for (int k = 0; k < ZB_M_NUM_REWARD_TERMS; ++k) ST(ZB_M_EP_SUMS + k) = 0.f;
  if (init) {
#pragma unroll
    for (int l = 0; l < NL; ++l) { ST(ZB_M_LINK_MU + l) = cfg.friction; ST(ZB_M_LINK_MU_D + l) = cfg.friction_dynamic; }
  }
#undef ST
}

// the observation of the current state (reset(): ObservationManager.compute after _reset_idx);
// noise from this call's stream
__global__ void zb_m_observe_kernel(const zb_model* __restrict__ mg, zb_task_cfg cfg, int N, const float* __restrict__ st,
                                    float* __restrict__ obs, const Counters* __restrict__ cnt, uint64_t seed) {
  MP m = to_mp(mg);
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= N) return;
  Phys p;
  load_phys(st, N, i, p);
  Kin k;
  fk(m, p, k);
  float bp[3], bq[4];
  link_pose(m, k, m->base_link, bp, bq);
  const float cmd[3] = {st[(size_t)ZB_M_COMMANDS * N + i], st[(size_t)(ZB_M_COMMANDS + 1) * N + i],
                        st[(size_t)(ZB_M_COMMANDS + 2) * N + i]};
  float a_obs[ND];
#pragma unroll
  for (int a = 0; a < ND; ++a) a_obs[a] = st[(size_t)(ZB_M_ACTIONS + a) * N + i];
  m_write_obs(m, cfg, env_hash(seed, cnt->calls, i), bq, cmd, p, a_obs, obs + (size_t)i * ZB_M_OBS_DIM);
}

// Episode log finalisation, curricula and the full-reset episode_length_buf draw (v2.py:418-422);
// leaves the accumulator zeroed for the next launch. Single workgroup (grid-strided over envs).
// The counters (RNG stream position, common_step_counter, curriculum state) live on the device so
// that a captured graph of zb_step advances them on every replay. Reset-mode events in the
// reference's order (v4 EventCfg 268-439): the episode log and the range-curriculum buffers
// (_reset_idx before the events), my_curriculum (one stage per call with resets once
// common_step_counter >= stage_steps[next]), range_curriculum (v4: widen the command ranges when
// the buffered tracking rewards exceed 85 % of their weight). New weights / ranges apply from the
// next step (the reference applies the reset-event ones to the commands it resamples in the same
// call). The manager's lin_vel_cmd_levels is exact: the reset envs' commands are
// redrawn here when it fires.
__device__ __forceinline__ void finalize_body(int N, float* __restrict__ st, float* __restrict__ acc,
                                              const FinArgs& fa, int force_full, int reset_counts, int is_step,
                                              const zb_task_cfg& cfg, float* __restrict__ obs,
                                              const uint8_t* __restrict__ term, const uint8_t* __restrict__ trunc,
                                              float* sh) {
  float* const log_means = fa.log_means;
  int32_t* const log_counts = fa.log_counts;
  float* const user_means = fa.user_means;
  int32_t* const user_counts = fa.user_counts;
  const float episode_s = fa.episode_s;
  const uint64_t seed = fa.seed;
  Counters* const cnt = fa.cnt;
  const int ep_len_row = fa.ep_len_row;
  const uint64_t ctr = cnt->calls;
  const uint64_t steps = cnt->steps + (is_step ? 1 : 0);
  // fold the accumulator slots (acc_slot): 8 groups of 8 slots x ACC_STRIDE entries, one
  // thread per (group, entry), which also clears what it read; then a shared sum of the groups.
  constexpr int FG = FIN_FG, FS = ACC_SLOTS / FG;
  float* const acc_part = sh;                     // [FG][ACC_STRIDE]
  float* const acc_sum = sh + FG * ACC_STRIDE;    // [ACC]
  for (int x = threadIdx.x; x < FG * ACC_STRIDE; x += blockDim.x) {
    const int g = x / ACC_STRIDE, t = x % ACC_STRIDE;
    float v[FS];
#pragma unroll
    for (int k = 0; k < FS; ++k) v[k] = acc[(g * FS + k) * ACC_STRIDE + t];
#pragma unroll
    for (int k = 0; k < FS; ++k) acc[(g * FS + k) * ACC_STRIDE + t] = 0.f;
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < FS; ++k) sum += v[k];
    acc_part[g * ACC_STRIDE + t] = sum;
  }
  __syncthreads();
  for (int x = threadIdx.x; x < ACC; x += blockDim.x) {
    float v = 0.f;
#pragma unroll
    for (int g = 0; g < FG; ++g) v += acc_part[g * ACC_STRIDE + x];
    acc_sum[x] = v;
  }
  __syncthreads();
  const float nres = acc_sum[ACC_NRES];
  const bool full = force_full || nres == (float)N;
  __syncthreads();
  if (threadIdx.x == 0) {
    cnt->steps = steps;
    cnt->changed = 0;
    if (nres > 0.f) {
      float v[ZB_LOG_LEN];
#pragma unroll
      for (int t = 0; t < ZB_MAX_REWARD_TERMS; ++t) v[t] = acc_sum[t] / nres / episode_s;
      v[16] = (float)cnt->stage;  // logged before the events run (v4.py:952-957)
      v[17] = cnt->vel[0];
      v[18] = cnt->vel[1];
      v[19] = cnt->yaw[0];
      if (cfg.task == ZB_TASK_MANAGER_V0) {
        // lin_vel_cmd_levels (curriculums.py:47-74) runs first in _reset_idx; it widens the
        // velocity ranges by +-delta when the mean episodic tracking reward / 20 s of the reset envs
        // exceeds 0.8 x its weight, on calls where common_step_counter % max_episode_length == 0
        if (cfg.range_period_steps > 0 && steps % (uint64_t)cfg.range_period_steps == 0 &&
            v[ZB_M_R_TRACK_LIN_VEL_XY] > cfg.stage_scales[0][ZB_M_R_TRACK_LIN_VEL_XY] * cfg.range_threshold) {
          cnt->vel[0] = clampf(cnt->vel[0] - cfg.range_delta, cfg.range_limit_vel[0], cfg.range_limit_vel[1]);
          cnt->vel[1] = clampf(cnt->vel[1] + cfg.range_delta, cfg.range_limit_vel[0], cfg.range_limit_vel[1]);
          cnt->yaw[0] = clampf(cnt->yaw[0] - cfg.range_delta, cfg.range_limit_yaw[0], cfg.range_limit_yaw[1]);
          cnt->yaw[1] = clampf(cnt->yaw[1] + cfg.range_delta, cfg.range_limit_yaw[0], cfg.range_limit_yaw[1]);
          cnt->changed = 1;
        }
        v[16] = cnt->vel[1];             // Curriculum/lin_vel_cmd_levels (the state after compute)
        v[17] = acc_sum[ACC_MET0] / nres;    // Metrics/base_velocity/error_vel_xy
        v[18] = acc_sum[ACC_MET1] / nres;    // Metrics/base_velocity/error_vel_yaw
        v[19] = 0.f;
      }
#pragma unroll
      for (int t = 0; t < ZB_LOG_LEN; ++t) {
        log_means[t] = v[t];
        if (user_means) user_means[t] = v[t];
      }
      const int32_t c[ZB_LOG_COUNTS] = {reset_counts ? 0 : (int32_t)acc_sum[ACC_DIED],
                                        reset_counts ? 0 : (int32_t)acc_sum[ACC_TOUT],
                                        reset_counts ? 0 : (int32_t)acc_sum[ACC_TERM2], 0};
#pragma unroll
      for (int k = 0; k < ZB_LOG_COUNTS; ++k) {
        log_counts[k] = c[k];
        if (user_counts) user_counts[k] = c[k];
      }
      if (cfg.task == ZB_TASK_WALKING_V4) {  // curriculum_*_reward_buffer.append (v4.py:941-944)
        cnt->ring_vel[cnt->ring_head] = v[ZB_V4_R_TRACK_LIN_VEL_X];
        cnt->ring_yaw[cnt->ring_head] = v[ZB_V4_R_TRACK_HEADING_YAW];
        cnt->ring_head = (cnt->ring_head + 1) % ZB_V4_RING;
        cnt->ring_n = min(cnt->ring_n + 1, ZB_V4_RING);
      }
      // my_curriculum
      const int s0 = cnt->stage;
      if (s0 + 1 < cfg.num_stages && s0 + 1 < ZB_MAX_STAGES && steps >= (uint64_t)cfg.stage_steps[s0 + 1]) {
        cnt->stage = s0 + 1;
        cnt->prob_pos = cfg.stage_prob_pos[s0 + 1];
      }
      // range_curriculum (v4.py:201-265)
      if (cfg.task == ZB_TASK_WALKING_V4 && cnt->ring_n >= cfg.range_min_buffer && cfg.range_period_steps > 0 &&
          steps >= (uint64_t)cfg.range_start_steps && steps % (uint64_t)cfg.range_period_steps == 0) {
        float mv = 0.f, my = 0.f;
        for (int k = 0; k < cnt->ring_n; ++k) { mv += cnt->ring_vel[k]; my += cnt->ring_yaw[k]; }
        mv /= (float)cnt->ring_n;
        my /= (float)cnt->ring_n;
        const int sg = cnt->stage;
        if (mv > cfg.stage_scales[sg][ZB_V4_R_TRACK_LIN_VEL_X] * cfg.range_threshold) {
          cnt->vel[0] = clampf(cnt->vel[0] - cfg.range_delta, cfg.range_limit_vel[0], cfg.range_limit_vel[1]);
          cnt->vel[1] = clampf(cnt->vel[1] + cfg.range_delta, cfg.range_limit_vel[0], cfg.range_limit_vel[1]);
        }
        if (my > cfg.stage_scales[sg][ZB_V4_R_TRACK_HEADING_YAW] * cfg.range_threshold) {
          cnt->yaw[0] = clampf(cnt->yaw[0] - cfg.range_delta, cfg.range_limit_yaw[0], cfg.range_limit_yaw[1]);
          cnt->yaw[1] = clampf(cnt->yaw[1] + cfg.range_delta, cfg.range_limit_yaw[0], cfg.range_limit_yaw[1]);
        }
      }
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) cnt->calls = ctr + 1;
  // the caller's per-step log accumulator (the PPO runner's mean over a rollout of extras["log"]): every
  // step adds the current values, those of this step if it had resets, else the last ones (persistent)
  if (is_step && fa.user_acc && threadIdx.x < ZB_LOG_LEN + ZB_LOG_COUNTS)
    fa.user_acc[threadIdx.x] += threadIdx.x < ZB_LOG_LEN ? log_means[threadIdx.x]
                                                         : (float)log_counts[threadIdx.x - ZB_LOG_LEN];
  // lin_vel_cmd_levels widened the ranges in this step: the reference's curriculum runs before the
  // command manager resamples the reset envs, so their commands (and the metrics / observations
  // that read them) are redrawn from the same draws with the new ranges (rare: at most once per
  // max_episode_length steps, so one workgroup does it)
  if (obs && cnt->changed)
    for (int i = threadIdx.x; i < N; i += blockDim.x)
      if (term[i] || trunc[i]) m_fixup_env(cfg, N, st, obs, cnt, env_hash(seed, ctr, i), i);
  if (full && cfg.task != ZB_TASK_MANAGER_V0)  // ManagerBasedRLEnv has no full-reset draw
    for (int i = threadIdx.x; i < N; i += blockDim.x) {
      const uint64_t h = hash64(seed ^ hash64(ctr * 0x100000001B3ull + (uint64_t)i));
      st[(size_t)ep_len_row * N + i] = (float)(int)(h % (uint64_t)cfg.max_episode_length);
    }
}

__global__ void zb_finalize_kernel(int N, float* __restrict__ st, float* __restrict__ acc,
                                   float* __restrict__ log_means, int32_t* __restrict__ log_counts,
                                   float* __restrict__ user_means, int32_t* __restrict__ user_counts, float episode_s,
                                   uint64_t seed, Counters* __restrict__ cnt, int force_full, int reset_counts,
                                   int is_step, int ep_len_row, zb_task_cfg cfg, float* __restrict__ obs,
                                   const uint8_t* __restrict__ term, const uint8_t* __restrict__ trunc,
                                   float* __restrict__ user_acc) {
  __shared__ float sh[FIN_FG * ACC_STRIDE + ACC];
  const FinArgs fa = {log_means, log_counts, user_means, user_counts, episode_s, seed, cnt, ep_len_row, user_acc};
  finalize_body(N, st, acc, fa, force_full, reset_counts, is_step, cfg, obs, term, trunc, sh);
}


}  // namespace

// =========================================================================== C ABI
#ifndef ZB_OCC1_DEFAULT
#define ZB_OCC1_DEFAULT 1
#endif
struct zb_sim {
  int device;
  int n;
  uint64_t seed;
  int task;           // ZB_TASK_*
  int state_dim;      // ZB_STATE_DIM / ZB_SU_STATE_DIM
  Counters* d_cnt;    // device counters (graph-replay safe)
  zb_task_cfg cfg;
  zb_model* d_model;
  float4* d_links;  // per-link collision table [NL][LINK4] (detect)
  float* d_state;
  float* d_wc = nullptr;  // persistent self-contact cache: ZB_WARM_ROWS x n
  float* d_acc;
  float* d_log_means;
  int32_t* d_log_counts;
  float* u_log_means = nullptr;     // optional caller buffers (zb_set_log_buffers)
  int32_t* u_log_counts = nullptr;
  float* u_log_acc = nullptr;       // optional caller accumulator (zb_set_log_accumulator)
  int64_t* u_done = nullptr;        // optional caller done buffer (zb_set_done_buffer)
  // ZB_DIAG_NO_FINALIZE=1 (diagnostic only, wrong results: no episode log, no full-reset draw, no
  // step counter): zb_step skips the finalize launch, to measure what that launch and its kernel
  // boundary cost per step
  bool diag_no_finalize = false;
  // optional per-launch timing of zb_step_kernel (hipEvents on the launch stream)
  int prof_max = 0, prof_n = 0;
  int prof_stride = 1, prof_seen = 0;  // time every prof_stride-th launch (zb_profile_stride)
  hipEvent_t* prof_ev = nullptr;
  bool occ1 = false;   // step kernels with one wave per SIMD (kOcc = 1; ZB_OCC1)
};

static thread_local char g_err[512] = "";

static int set_err(int code, const char* what, hipError_t e) {
  snprintf(g_err, sizeof(g_err), "%s: %s", what, e == hipSuccess ? "invalid argument" : hipGetErrorString(e));
  return code;
}

#define HIPCHK(x, what)                                   \
  do {                                                    \
    hipError_t e_ = (x);                                  \
    if (e_ != hipSuccess) return set_err(-2, what, e_);   \
  } while (0)

static int launch_check(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return set_err(-3, what, e);
  return 0;
}

// a step-kernel launch; with events (zb_profile_begin) the dispatch itself records the kernel's start
// and end (hipExtLaunchKernelGGL): the in-process time then is the kernel's own, as rocprofv3 reports
// it, without the latency of separate event packets
template <typename F, typename... Args>
void zb_launch(F kernel, int blocks, hipStream_t s, hipEvent_t e0, hipEvent_t e1, Args... args) {
  if (e0)
    hipExtLaunchKernelGGL(kernel, dim3(blocks), dim3(WGT), 0, s, e0, e1, 0, args...);
  else
    hipLaunchKernelGGL(kernel, dim3(blocks), dim3(WGT), 0, s, args...);
}

extern "C" {

const char* zb_last_error(void) { return g_err; }

int zb_num_envs(zb_handle h) { return h ? h->n : -1; }

int zb_create(const zb_model* m, const zb_task_cfg* c, int num_envs, int hip_device, uint64_t seed, zb_handle* out) {
  if (!m || !c || !out || num_envs <= 0) return set_err(-1, "zb_create", hipSuccess);
  for (int l = 0; l < NL; ++l)
    if (m->link_body[l] != link_body(l)) return set_err(-1, "zb_create: model topology != compiled ZBOT-6 chain", hipSuccess);
  if ((m->base_link != 6 && !(c->task == ZB_TASK_MANAGER_V0 && m->base_link == 5)) || m->foot_links[0] != 0 ||
      m->foot_links[1] != 11)
    return set_err(-1, "zb_create: unexpected base/feet link indices", hipSuccess);
  for (int k = 0; k < 10; ++k)
    if (m->undesired_links[k] != k + 1) return set_err(-1, "zb_create: unexpected undesired link set", hipSuccess);
  {
    int np = 0;
    for (int a = 0; a < NL; ++a)
      for (int b = a + 2; b < NL; ++b) {
        if (np >= m->num_self_pairs || m->self_pairs[np][0] != a || m->self_pairs[np][1] != b)
          return set_err(-1, "zb_create: self-collision pair list != compiled list", hipSuccess);
        ++np;
      }
    if (np != m->num_self_pairs) return set_err(-1, "zb_create: self-collision pair count", hipSuccess);
  }
  if (c->decimation < 1 || c->decimation > MAXSUB || c->solver_iterations < 0 || c->solver_mode < 0 ||
      c->solver_mode > 3 || (c->solver_mode >= 1 && c->solver_iterations < 1) ||
      (c->solver_mode >= 2 && c->task != ZB_TASK_WALKING_V2 && c->task != ZB_TASK_STANDUP_V0) ||
      c->self_manifold < 0 || c->self_manifold > 3 ||
      (c->self_manifold == 3 && c->task != ZB_TASK_WALKING_V2 && c->task != ZB_TASK_STANDUP_V0))
    return set_err(-1, "zb_create: cfg (decimation 1..8, solver_iterations >= 0, solver_mode 0..3, iterations "
                       ">= 1 from mode 1; modes 2, 3 for walking v2 and stand-up; self_manifold 0..3, 3 for "
                       "walking v2 and stand-up)",
                   hipSuccess);
  if (c->task != ZB_TASK_WALKING_V2 && c->task != ZB_TASK_STANDUP_V0 && c->task != ZB_TASK_WALKING_V4 &&
      c->task != ZB_TASK_MANAGER_V0)
    return set_err(-1, "zb_create: unknown task", hipSuccess);
  if (c->num_stages < 1 || c->num_stages > ZB_MAX_STAGES) return set_err(-1, "zb_create: num_stages", hipSuccess);
  if (c->task == ZB_TASK_WALKING_V2)  // a weighted term must be active (a zero-initialised reward_active would
    for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t)  // freeze its buffers silently; include/zbot.h)
      if (c->reward_scales[t] != 0.f && !((c->reward_active >> t) & 1u))
        return set_err(-1, "zb_create: reward term with a non-zero scale but its reward_active bit clear", hipSuccess);
  if (c->task == ZB_TASK_STANDUP_V0 && c->center_z_period < 1) return set_err(-1, "zb_create: center_z_period", hipSuccess);
  HIPCHK(hipSetDevice(hip_device), "hipSetDevice");
  zb_sim* h = new zb_sim();
  h->device = hip_device;
  h->n = num_envs;
  h->seed = seed;
  h->task = c->task;
  h->state_dim = c->task == ZB_TASK_STANDUP_V0 ? ZB_SU_STATE_DIM
                 : c->task == ZB_TASK_WALKING_V4 ? ZB_V4_STATE_DIM
                 : c->task == ZB_TASK_MANAGER_V0 ? ZB_M_STATE_DIM : ZB_STATE_DIM;
  h->d_cnt = nullptr;
  h->cfg = *c;
  HIPCHK(hipMalloc(&h->d_model, sizeof(zb_model)), "hipMalloc model");
  HIPCHK(hipMalloc(&h->d_state, sizeof(float) * (size_t)h->state_dim * num_envs), "hipMalloc state");
  HIPCHK(hipMalloc(&h->d_acc, sizeof(float) * ACC_SLOTS * ACC_STRIDE), "hipMalloc acc");
  HIPCHK(hipMalloc(&h->d_cnt, sizeof(Counters)), "hipMalloc counters");
  {
    // one wave per SIMD at <= 4096 envs (<= one wave per SIMD anyway): ZB_OCC1=0/1 overrides (only
    // an explicit "1" / "0": an empty value or "false" does not)
    const char* oc = getenv("ZB_OCC1");
    const int oc_on = oc && oc[0] == '1' && oc[1] == 0, oc_off = oc && oc[0] == '0' && oc[1] == 0;
    h->occ1 = oc_on || (!oc_off && ZB_OCC1_DEFAULT && num_envs <= 4096);
    const char* nf = getenv("ZB_DIAG_NO_FINALIZE");
    h->diag_no_finalize = nf && nf[0] == '1' && nf[1] == 0;
  }
  {
    Counters c0;
    memset(&c0, 0, sizeof(c0));
    c0.vel[0] = c->cmd_vel_range[0]; c0.vel[1] = c->cmd_vel_range[1];
    c0.yaw[0] = c->cmd_yaw_range[0]; c0.yaw[1] = c->cmd_yaw_range[1];
    c0.prob_pos = c->stage_prob_pos[0];
    HIPCHK(hipMemcpy(h->d_cnt, &c0, sizeof(Counters), hipMemcpyHostToDevice), "hipMemcpy counters");
  }
  HIPCHK(hipMalloc(&h->d_log_means, sizeof(float) * ZB_LOG_LEN), "hipMalloc log");
  HIPCHK(hipMalloc(&h->d_log_counts, sizeof(int32_t) * ZB_LOG_COUNTS), "hipMalloc log");
  HIPCHK(hipMemcpy(h->d_model, m, sizeof(zb_model), hipMemcpyHostToDevice), "hipMemcpy model");
  {
    float4 tab[LNK4];
    memset(tab, 0, sizeof(tab));
    for (int l = 0; l < NL; ++l) {
      float4* t = tab + l * LINK4;
      t[0] = make_float4(m->link_bound[l][0], m->link_bound[l][1], m->link_bound[l][2], m->link_bound[l][3]);
      for (int ci = 0; ci < 2; ++ci)
        for (int v = 0; v < 3; ++v) {
          const float* c = m->link_circle[l][ci] + 3 * v;
          // C.w = 1: a mated face duplicating a lower link's circle (ground detection skips it)
          t[1 + 3 * ci + v] = make_float4(c[0], c[1], c[2], v == 0 && ((m->link_circle_dup[l] >> ci) & 1) ? 1.f : 0.f);
        }
      // self-collision core circles (kCoreM into the shape along each circle's normal, radius
      // r - kCoreM; the same rule as the oracle's load_mdl): {centre, semi-axis scale}
      double mid[3], rad = 0.0;
      for (int a = 0; a < 3; ++a) mid[a] = 0.5 * ((double)m->link_circle[l][0][a] + m->link_circle[l][1][a]);
      for (int ci = 0; ci < 2; ++ci) {
        const float* c = m->link_circle[l][ci];
        const float* o = m->link_circle[l][1 - ci];
        double n[3] = {(double)c[4] * c[8] - (double)c[5] * c[7], (double)c[5] * c[6] - (double)c[3] * c[8],
                       (double)c[3] * c[7] - (double)c[4] * c[6]};
        const double nn = sqrt(n[0] * n[0] + n[1] * n[1] + n[2] * n[2]);
        const double r = sqrt((double)c[3] * c[3] + (double)c[4] * c[4] + (double)c[5] * c[5]);
        const double to = n[0] * (o[0] - c[0]) + n[1] * (o[1] - c[1]) + n[2] * (o[2] - c[2]);
        const double sg = to < 0.0 ? -1.0 : 1.0;
        t[7 + ci] = make_float4((float)(c[0] + sg * kCoreM * n[0] / nn), (float)(c[1] + sg * kCoreM * n[1] / nn),
                                (float)(c[2] + sg * kCoreM * n[2] / nn), (float)((r - kCoreM) / r));
        const double dc = sqrt((c[0] - mid[0]) * (c[0] - mid[0]) + (c[1] - mid[1]) * (c[1] - mid[1]) +
                               (c[2] - mid[2]) * (c[2] - mid[2]));
        rad = fmax(rad, dc + r);
      }
      // bounding sphere of the whole shape
      t[9] = make_float4((float)mid[0], (float)mid[1], (float)mid[2], (float)(rad + 1e-6));
      // self-collision broadphase: the core hull lies in the capsule of its two core circle centres
      // with the larger core radius (+ 1 um)
      {
        double rc = 0.0;
        for (int ci = 0; ci < 2; ++ci) {
          const float* c = m->link_circle[l][ci];
          rc = fmax(rc, sqrt((double)c[3] * c[3] + (double)c[4] * c[4] + (double)c[5] * c[5]) - kCoreM);
        }
        t[2].w = (float)(rc + 1e-6);
      }
    }
    for (int j = 0; j < ND; ++j) {
      float4* t = tab + JT_OFF + j * 5;
      const float* r = m->joint_parent_rot[j];
      t[0] = make_float4(r[0], r[1], r[2], r[3]);
      t[1] = make_float4(m->joint_parent_pos[j][0], m->joint_parent_pos[j][1], m->joint_parent_pos[j][2], 0.f);
      t[2] = make_float4(m->joint_child_pos[j][0], m->joint_child_pos[j][1], m->joint_child_pos[j][2], 0.f);
      const float* c = m->joint_child_rot[j];
      t[3] = make_float4(c[0], c[1], c[2], c[3]);
      const float w = r[0], x = r[1], y = r[2], z = r[3];  // third column of R(jpr)
      t[4] = make_float4(2.f * (x * z + w * y), 2.f * (y * z - w * x), 1.f - 2.f * (x * x + y * y), 0.f);
    }
    for (int b = 0; b < NB; ++b) {
      float4* t = tab + BT_OFF + b * 3;
      const float* I = m->body_inertia[b];
      t[0] = make_float4(m->body_com[b][0], m->body_com[b][1], m->body_com[b][2], m->body_mass[b]);
      t[1] = make_float4(I[0], I[1], I[2], I[3]);
      t[2] = make_float4(I[4], I[5], 0.f, 0.f);
    }
    int* pc = reinterpret_cast<int*>(tab + NL * LINK4);
    for (int p = 0; p < m->num_self_pairs; ++p) pc[p] = 16 * m->self_pairs[p][0] + m->self_pairs[p][1];
    HIPCHK(hipMalloc(&h->d_links, sizeof(tab)), "hipMalloc links");
    HIPCHK(hipMemcpy(h->d_links, tab, sizeof(tab), hipMemcpyHostToDevice), "hipMemcpy links");
  }
  HIPCHK(hipMemset(h->d_state, 0, sizeof(float) * (size_t)h->state_dim * num_envs), "hipMemset state");
  HIPCHK(hipMemset(h->d_log_means, 0, sizeof(float) * ZB_LOG_LEN), "hipMemset log");
  HIPCHK(hipMemset(h->d_log_counts, 0, sizeof(int32_t) * ZB_LOG_COUNTS), "hipMemset log");
  HIPCHK(hipMemset(h->d_acc, 0, sizeof(float) * ACC_SLOTS * ACC_STRIDE), "hipMemset acc");
  // start at the default pose (ep_len 0, as after construction; reset() randomises it)
  zb_derive_kernel<<<1, 1>>>(h->d_model, h->d_links);
  int rc = launch_check("zb_derive_kernel");
  if (rc) return rc;
  if (h->task == ZB_TASK_STANDUP_V0) {
    zb_su_friction_kernel<<<(num_envs * NL + 255) / 256, 256>>>(num_envs, h->d_state, nullptr, c->friction, ZB_SU_LINK_MU);
    rc = launch_check("zb_su_friction_kernel");
    if (rc) return rc;
    zb_su_friction_kernel<<<(num_envs * NL + 255) / 256, 256>>>(num_envs, h->d_state, nullptr, c->friction_dynamic,
                                                                ZB_SU_LINK_MU_D);
    rc = launch_check("zb_su_friction_kernel");
    if (rc) return rc;
    // the construction-time reset draws its poses at RNG position 0; later calls start at 1
    zb_su_reset_kernel<<<(num_envs + 255) / 256, 256>>>(h->d_model, h->cfg, num_envs, h->d_state, nullptr, num_envs,
                                                       h->d_acc, h->d_cnt, h->seed);
    rc = launch_check("zb_su_reset_kernel");
    if (rc) return rc;
    const uint64_t one = 1;
    HIPCHK(hipMemcpy(&h->d_cnt->calls, &one, sizeof(one), hipMemcpyHostToDevice), "hipMemcpy counters");
  } else if (h->task == ZB_TASK_WALKING_V4) {
    // construction: reset events at RNG position 0 (+ interval timers); later calls start at 1
    zb_v4_reset_kernel<<<(num_envs + 255) / 256, 256>>>(h->d_model, h->d_links, h->cfg, num_envs, h->d_state, nullptr,
                                                       num_envs, h->d_acc, h->d_cnt, h->seed, 1);
    rc = launch_check("zb_v4_reset_kernel");
    if (rc) return rc;
    const uint64_t one = 1;
    HIPCHK(hipMemcpy(&h->d_cnt->calls, &one, sizeof(one), hipMemcpyHostToDevice), "hipMemcpy counters");
  } else if (h->task == ZB_TASK_MANAGER_V0) {
    // construction: ManagerBasedRLEnv.__init__ -> load_managers + reset events at RNG position 0
    // (friction default fill; the startup material event overwrites it); later calls start at 1
    zb_m_reset_kernel<<<(num_envs + 255) / 256, 256>>>(h->d_model, h->d_links, h->cfg, num_envs, h->d_state, nullptr,
                                                      num_envs, h->d_acc, h->d_cnt, h->seed, 1);
    rc = launch_check("zb_m_reset_kernel");
    if (rc) return rc;
    const uint64_t one = 1;
    HIPCHK(hipMemcpy(&h->d_cnt->calls, &one, sizeof(one), hipMemcpyHostToDevice), "hipMemcpy counters");
  } else {
    // construction: the spawn pose is the default pose, so the latch reads the default feet
    zb_reset_kernel<<<(num_envs + 255) / 256, 256>>>(h->d_model, h->d_links, num_envs, h->d_state, nullptr, num_envs,
                                                      h->d_acc, 1);
    rc = launch_check("zb_reset_kernel");
  }
  if (rc) return rc;
  HIPCHK(hipMemset(h->d_acc, 0, sizeof(float) * ACC_SLOTS * ACC_STRIDE), "hipMemset acc");
  {
    HIPCHK(hipMalloc(&h->d_wc, sizeof(float) * ZB_WARM_ROWS * (size_t)num_envs), "hipMalloc contact cache");
    zb_wc_fill_kernel<<<(num_envs * ZB_WARM_ROWS + 255) / 256, 256>>>(num_envs, h->d_wc, nullptr, num_envs);
    rc = launch_check("zb_wc_fill_kernel");
    if (rc) return rc;
  }
  HIPCHK(hipDeviceSynchronize(), "zb_create sync");
  *out = h;
  return 0;
}

static void prof_free(zb_handle h) {
  for (int k = 0; k < 2 * h->prof_max; ++k) (void)hipEventDestroy(h->prof_ev[k]);
  delete[] h->prof_ev;
  h->prof_ev = nullptr;
  h->prof_max = h->prof_n = 0;
}

int zb_profile_begin(zb_handle h, int max_launches) {
  if (!h || max_launches < 0) return set_err(-1, "zb_profile_begin", hipSuccess);
  prof_free(h);
  h->prof_ev = new hipEvent_t[2 * (size_t)max_launches];
  for (int k = 0; k < 2 * max_launches; ++k) HIPCHK(hipEventCreate(&h->prof_ev[k]), "hipEventCreate");
  h->prof_max = max_launches;
  h->prof_n = 0;
  h->prof_seen = 0;
  return 0;
}

int zb_profile_stride(zb_handle h, int stride) {
  if (!h || stride < 1) return set_err(-1, "zb_profile_stride", hipSuccess);
  h->prof_stride = stride;
  return 0;
}

int zb_profile_end(zb_handle h, float* total_ms, int* count) {
  if (!h || !total_ms || !count) return set_err(-1, "zb_profile_end", hipSuccess);
  float tot = 0.f;
  for (int k = 0; k < h->prof_n; ++k) {
    HIPCHK(hipEventSynchronize(h->prof_ev[2 * k + 1]), "hipEventSynchronize");
    float ms = 0.f;
    HIPCHK(hipEventElapsedTime(&ms, h->prof_ev[2 * k], h->prof_ev[2 * k + 1]), "hipEventElapsedTime");
    tot += ms;
  }
  *total_ms = tot;
  *count = h->prof_n;
  prof_free(h);
  return 0;
}

// Diagnostic build only (-DZB_STAMPS): the phase cycles of the slowest wave since the last reset.
int zb_read_stamps_slowest(uint64_t* out16) {
#ifdef ZB_STAMPS
  unsigned long long tmp[NSTAMP];
  HIPCHK(hipMemcpyFromSymbol(tmp, HIP_SYMBOL(g_stamp_slowest), sizeof(tmp)), "hipMemcpyFromSymbol");
  for (int k = 0; k < 16; ++k) out16[k] = k < NSTAMP ? tmp[k] : 0;
  return 0;
#else
  (void)out16;
  return set_err(-1, "zb_read_stamps_slowest: library built without -DZB_STAMPS", hipSuccess);
#endif
}

// Diagnostic build only (-DZB_STAMPS): per-phase cycle sums over all waves since the last call.
int zb_read_stamp_hist(uint64_t* out136) {
  uint64_t* out128 = out136;
#ifdef ZB_STAMPS
  unsigned long long tmp[kCapCounters + 8];
  HIPCHK(hipMemcpyFromSymbol(tmp, HIP_SYMBOL(g_stamp_hist), sizeof(tmp)), "hipMemcpyFromSymbol");
  for (int k = 0; k < kCapCounters + 8; ++k) out128[k] = tmp[k];
  unsigned long long z[kCapCounters + 8] = {0};
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamp_hist), z, sizeof(z)), "hipMemcpyToSymbol");
  return 0;
#else
  (void)out128;
  return set_err(-1, "zb_read_stamp_hist: library built without -DZB_STAMPS", hipSuccess);
#endif
}
// Diagnostic build only (-DZB_STAMPS): per workgroup of the latest step launch {start, end}
// (s_memrealtime ticks, 100 MHz) and its 13 phase cycle counts; n workgroups.
int zb_read_wave_times(uint64_t* out, int n) {
#ifdef ZB_STAMPS
  if (!out || n < 0 || n > kMaxWaveRecs) return set_err(-1, "zb_read_wave_times", hipSuccess);
  HIPCHK(hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wave_rec), sizeof(unsigned long long) * kWaveRec * (size_t)n),
         "hipMemcpyFromSymbol");
  return 0;
#else
  (void)out; (void)n;
  return set_err(-1, "zb_read_wave_times: library built without -DZB_STAMPS", hipSuccess);
#endif
}
int zb_read_stamps(uint64_t* out16) {
#ifdef ZB_STAMPS
  unsigned long long tmp[NSTAMP];
  HIPCHK(hipMemcpyFromSymbol(tmp, HIP_SYMBOL(g_stamps), sizeof(tmp)), "hipMemcpyFromSymbol");
  for (int k = 0; k < 16; ++k) out16[k] = k < NSTAMP ? tmp[k] : 0;
  unsigned long long z[NSTAMP] = {0};
  HIPCHK(hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), z, sizeof(z)), "hipMemcpyToSymbol");
  return 0;
#else
  (void)out16;
  return set_err(-1, "zb_read_stamps: library built without -DZB_STAMPS", hipSuccess);
#endif
}

void zb_destroy(zb_handle h) {
  if (!h) return;
  prof_free(h);
  (void)hipSetDevice(h->device);
  (void)hipFree(h->d_model);
  (void)hipFree(h->d_links);
  (void)hipFree(h->d_state);
  (void)hipFree(h->d_wc);
  (void)hipFree(h->d_acc);
  (void)hipFree(h->d_cnt);
  (void)hipFree(h->d_log_means);
  (void)hipFree(h->d_log_counts);
  delete h;
}

// episode-log divisor: walking divides the summed episode sums by the 20 s episode (v2.py:446),
// standup already divided each env's sums by its own duration (standup.py:653-659)
static float log_episode_s(zb_handle h) {
  // (the manager's RewardManager.reset divides by max_episode_length_s too)
  return h->task == ZB_TASK_WALKING_V2 || h->task == ZB_TASK_MANAGER_V0
             ? h->cfg.sim_dt * h->cfg.decimation * h->cfg.max_episode_length
             : 1.f;
}

static int finalize(zb_handle h, hipStream_t s, int full, int reset_counts, int is_step, float* obs = nullptr,
                    const uint8_t* term = nullptr, const uint8_t* trunc = nullptr) {
  const int ep_row = h->task == ZB_TASK_STANDUP_V0   ? ZB_SU_EP_LEN
                     : h->task == ZB_TASK_WALKING_V4 ? ZB_V4_EP_LEN
                     : h->task == ZB_TASK_MANAGER_V0 ? ZB_M_EP_LEN
                                                     : ZB_S_EP_LEN;
  zb_finalize_kernel<<<1, 256, 0, s>>>(h->n, h->d_state, h->d_acc, h->d_log_means, h->d_log_counts, h->u_log_means,
                                       h->u_log_counts, log_episode_s(h), h->seed, h->d_cnt, full, reset_counts, is_step,
                                       ep_row, h->cfg, obs, term, trunc, h->u_log_acc);
  return launch_check("zb_finalize_kernel");
}

int zb_reset(zb_handle h, const int32_t* env_ids, int n, void* stream) {
  if (!h) return set_err(-1, "zb_reset", hipSuccess);
  hipStream_t s = (hipStream_t)stream;
  const int cnt = env_ids ? n : h->n;
  if (cnt <= 0) return 0;
  if (h->task == ZB_TASK_STANDUP_V0)
    zb_su_reset_kernel<<<(cnt + 255) / 256, 256, 0, s>>>(h->d_model, h->cfg, h->n, h->d_state, env_ids, cnt, h->d_acc,
                                                         h->d_cnt, h->seed);
  else if (h->task == ZB_TASK_WALKING_V4)
    zb_v4_reset_kernel<<<(cnt + 255) / 256, 256, 0, s>>>(h->d_model, h->d_links, h->cfg, h->n, h->d_state, env_ids, cnt,
                                                         h->d_acc, h->d_cnt, h->seed, 0);
  else if (h->task == ZB_TASK_MANAGER_V0)
    zb_m_reset_kernel<<<(cnt + 255) / 256, 256, 0, s>>>(h->d_model, h->d_links, h->cfg, h->n, h->d_state, env_ids, cnt,
                                                        h->d_acc, h->d_cnt, h->seed, 0);
  else
    zb_reset_kernel<<<(cnt + 255) / 256, 256, 0, s>>>(h->d_model, h->d_links, h->n, h->d_state, env_ids, cnt, h->d_acc,
                                                      h->cfg.reset_feet_refresh);
  int rc = launch_check("zb_reset_kernel");
  if (rc) return rc;
  if (h->d_wc) {
    zb_wc_fill_kernel<<<(cnt * ZB_WARM_ROWS + 255) / 256, 256, 0, s>>>(h->n, h->d_wc, env_ids, cnt);
    rc = launch_check("zb_wc_fill_kernel");
    if (rc) return rc;
  }
  return finalize(h, s, env_ids == nullptr || n == h->n, 1, 0);
}

int zb_step(zb_handle h, const float* actions, float* obs, float* reward, uint8_t* terminated, uint8_t* truncated,
            void* stream) {
  if (!h || !actions || !obs || !reward || !terminated || !truncated) return set_err(-1, "zb_step", hipSuccess);
  hipStream_t s = (hipStream_t)stream;
  const int blocks = (h->n + EPW - 1) / EPW;
  // (the event-recording dispatch adds ~5.7 us to a step: every prof_stride-th launch only)
  const bool prof = h->prof_n < h->prof_max && (h->prof_seen++ % h->prof_stride) == 0;
  hipEvent_t e0 = prof ? h->prof_ev[2 * h->prof_n] : nullptr, e1 = prof ? h->prof_ev[2 * h->prof_n + 1] : nullptr;
  const bool tgs = h->cfg.solver_mode >= 1, refresh = h->cfg.solver_mode >= 2;
  const bool one = h->occ1;
#define ZB_LAUNCH(K, ...)                                                                          \
  (tgs ? (one ? zb_launch(K<true, 1>, blocks, s, e0, e1, __VA_ARGS__) : zb_launch(K<true, 2>, blocks, s, e0, e1, __VA_ARGS__)) \
       : (one ? zb_launch(K<false, 1>, blocks, s, e0, e1, __VA_ARGS__) : zb_launch(K<false, 2>, blocks, s, e0, e1, __VA_ARGS__)))
  // solver_modes 2, 3 (the TGS refresh) and self_manifold 3 (the ruling-on-face manifold): walking v2
  // and stand-up only (zb_create); one wave per SIMD at <= 4096 envs as the default kernels (round 6:
  // the refresh's FK and row rebuild inside the sweeps spill at two-wave occupancy)
  const bool rf = h->cfg.self_manifold == 3;
#define ZB_LAUNCH_R(K, ...)                                                                        \
  (rf ? (refresh ? (one ? zb_launch(K<true, 1, true, true>, blocks, s, e0, e1, __VA_ARGS__)          \
                        : zb_launch(K<true, 2, true, true>, blocks, s, e0, e1, __VA_ARGS__))         \
                 : (tgs ? (one ? zb_launch(K<true, 1, false, true>, blocks, s, e0, e1, __VA_ARGS__)  \
                               : zb_launch(K<true, 2, false, true>, blocks, s, e0, e1, __VA_ARGS__)) \
                        : (one ? zb_launch(K<false, 1, false, true>, blocks, s, e0, e1, __VA_ARGS__) \
                               : zb_launch(K<false, 2, false, true>, blocks, s, e0, e1, __VA_ARGS__)))) \
      : refresh ? (one ? zb_launch(K<true, 1, true>, blocks, s, e0, e1, __VA_ARGS__)                 \
                       : zb_launch(K<true, 2, true>, blocks, s, e0, e1, __VA_ARGS__))                \
                : ZB_LAUNCH(K, __VA_ARGS__))
  if (h->task == ZB_TASK_STANDUP_V0)
    ZB_LAUNCH_R(zb_su_step_kernel, h->d_model, h->d_links, h->cfg, h->n, h->d_state, actions, obs, reward, terminated,
              truncated, h->u_done, h->d_acc, h->d_cnt, h->seed, h->d_wc);
  else if (h->task == ZB_TASK_WALKING_V4)
    ZB_LAUNCH(zb_v4_step_kernel, h->d_model, h->d_links, h->cfg, h->n, h->d_state, actions, obs, reward, terminated,
              truncated, h->u_done, h->d_acc, h->d_cnt, h->seed, h->d_wc);
  else if (h->task == ZB_TASK_MANAGER_V0)
    ZB_LAUNCH(zb_m_step_kernel, h->d_model, h->d_links, h->cfg, h->n, h->d_state, actions, obs, reward, terminated,
              truncated, h->u_done, h->d_acc, h->d_cnt, h->seed, h->d_wc);
  else
    ZB_LAUNCH_R(zb_step_kernel, h->d_model, h->d_links, h->cfg, h->n, h->d_state, actions, obs, reward, terminated,
              truncated, h->u_done, h->d_acc, h->d_wc);
#undef ZB_LAUNCH_R
#undef ZB_LAUNCH
  int rc = launch_check("zb_step_kernel");
  if (prof) ++h->prof_n;
  if (rc) return rc;
  if (h->diag_no_finalize) return 0;  // (diagnostic, DESIGN.md §7: the finalize launch's share of a step)
  return finalize(h, s, 0, 0, 1, obs, terminated, truncated);
}

int zb_observe(zb_handle h, float* obs, void* stream) {
  if (!h || !obs) return set_err(-1, "zb_observe", hipSuccess);
  if (h->task == ZB_TASK_STANDUP_V0)
    zb_su_observe_kernel<<<(h->n + 255) / 256, 256, 0, (hipStream_t)stream>>>(h->d_model, h->n, h->d_state, obs);
  else if (h->task == ZB_TASK_WALKING_V4)
    zb_v4_observe_kernel<<<(h->n + 255) / 256, 256, 0, (hipStream_t)stream>>>(h->d_model, h->n, h->d_state, obs);
  else if (h->task == ZB_TASK_MANAGER_V0)
    zb_m_observe_kernel<<<(h->n + 255) / 256, 256, 0, (hipStream_t)stream>>>(h->d_model, h->cfg, h->n, h->d_state, obs,
                                                                             h->d_cnt, h->seed);
  else
    zb_observe_kernel<<<(h->n + 255) / 256, 256, 0, (hipStream_t)stream>>>(h->d_model, h->n, h->d_state, obs);
  return launch_check("zb_observe_kernel");
}

int zb_state_dim(zb_handle h) { return h ? h->state_dim : -1; }

int zb_set_link_friction_sd(zb_handle h, const float* mu_static, const float* mu_dynamic, void* stream) {
  if (!h || !mu_static || !mu_dynamic) return set_err(-1, "zb_set_link_friction_sd", hipSuccess);
  if (h->task != ZB_TASK_STANDUP_V0 && h->task != ZB_TASK_MANAGER_V0)
    return set_err(-1, "zb_set_link_friction: per-link friction is a standup / manager task state", hipSuccess);
  const bool mgr = h->task == ZB_TASK_MANAGER_V0;
  zb_su_friction_kernel<<<(h->n * NL + 255) / 256, 256, 0, (hipStream_t)stream>>>(
      h->n, h->d_state, mu_static, 0.f, mgr ? ZB_M_LINK_MU : ZB_SU_LINK_MU);
  int rc = launch_check("zb_su_friction_kernel");
  if (rc) return rc;
  zb_su_friction_kernel<<<(h->n * NL + 255) / 256, 256, 0, (hipStream_t)stream>>>(
      h->n, h->d_state, mu_dynamic, 0.f, mgr ? ZB_M_LINK_MU_D : ZB_SU_LINK_MU_D);
  return launch_check("zb_su_friction_kernel");
}

int zb_set_link_friction(zb_handle h, const float* mu, void* stream) {
  return zb_set_link_friction_sd(h, mu, mu, stream);
}

int zb_read_curriculum(zb_handle h, int32_t* stage, int64_t* common_step_counter) {
  if (!h) return set_err(-1, "zb_read_curriculum", hipSuccess);
  Counters c;
  HIPCHK(hipMemcpy(&c, h->d_cnt, sizeof(Counters), hipMemcpyDeviceToHost), "hipMemcpy counters");
  if (stage) *stage = c.stage;
  if (common_step_counter) *common_step_counter = (int64_t)c.steps;
  return 0;
}

int zb_read_log(zb_handle h, float* term_means, int32_t* counts, void* stream) {
  if (!h) return set_err(-1, "zb_read_log", hipSuccess);
  hipStream_t s = (hipStream_t)stream;
  if (term_means)
    HIPCHK(hipMemcpyAsync(term_means, h->d_log_means, sizeof(float) * ZB_LOG_LEN, hipMemcpyDeviceToDevice, s),
           "hipMemcpyAsync log");
  if (counts)
    HIPCHK(hipMemcpyAsync(counts, h->d_log_counts, sizeof(int32_t) * ZB_LOG_COUNTS, hipMemcpyDeviceToDevice, s),
           "hipMemcpyAsync log");
  return 0;
}

int zb_set_log_buffers(zb_handle h, float* term_means, int32_t* counts) {
  if (!h || (!term_means) != (!counts)) return set_err(-1, "zb_set_log_buffers", hipSuccess);
  h->u_log_means = term_means;
  h->u_log_counts = counts;
  return 0;
}

int zb_set_done_buffer(zb_handle h, int64_t* dones) {
  if (!h) return set_err(-1, "zb_set_done_buffer", hipSuccess);
  h->u_done = dones;
  return 0;
}

int zb_set_log_accumulator(zb_handle h, float* acc) {
  if (!h) return set_err(-1, "zb_set_log_accumulator", hipSuccess);
  h->u_log_acc = acc;
  return 0;
}

int zb_get_state(zb_handle h, float* dst, void* stream) {
  if (!h || !dst) return set_err(-1, "zb_get_state", hipSuccess);
  HIPCHK(hipMemcpyAsync(dst, h->d_state, sizeof(float) * (size_t)h->state_dim * h->n, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream),
         "hipMemcpyAsync state");
  return 0;
}

int zb_set_state(zb_handle h, const float* src, void* stream) {
  if (!h || !src) return set_err(-1, "zb_set_state", hipSuccess);
  HIPCHK(hipMemcpyAsync(h->d_state, src, sizeof(float) * (size_t)h->state_dim * h->n, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream),
         "hipMemcpyAsync state");
  if (h->d_wc) {  // a new state: no warm start from the old one's contacts
    zb_wc_fill_kernel<<<(h->n * ZB_WARM_ROWS + 255) / 256, 256, 0, (hipStream_t)stream>>>(h->n, h->d_wc, nullptr, h->n);
    return launch_check("zb_wc_fill_kernel");
  }
  return 0;
}

int zb_get_contact_cache(zb_handle h, float* dst, void* stream) {
  if (!h || !dst || !h->d_wc) return set_err(-1, "zb_get_contact_cache", hipSuccess);
  HIPCHK(hipMemcpyAsync(dst, h->d_wc, sizeof(float) * ZB_WARM_ROWS * (size_t)h->n, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream),
         "hipMemcpyAsync contact cache");
  return 0;
}

int zb_set_contact_cache(zb_handle h, const float* src, void* stream) {
  if (!h || !src || !h->d_wc) return set_err(-1, "zb_set_contact_cache", hipSuccess);
  HIPCHK(hipMemcpyAsync(h->d_wc, src, sizeof(float) * ZB_WARM_ROWS * (size_t)h->n, hipMemcpyDeviceToDevice,
                        (hipStream_t)stream),
         "hipMemcpyAsync contact cache");
  return 0;
}

int zb_physics_substeps(zb_handle h, const float* targets, int nsub, float* net_force, float* applied_torque,
                        void* stream) {
  if (!h || !targets || nsub < 1) return set_err(-1, "zb_physics_substeps", hipSuccess);
  const int blocks = (h->n + EPW - 1) / EPW;
  const bool dr = h->task == ZB_TASK_STANDUP_V0 || h->task == ZB_TASK_MANAGER_V0, tgs = h->cfg.solver_mode >= 1;
  const bool refresh = h->cfg.solver_mode >= 2;
#define ZB_SUB(F, T, R) zb_substeps_kernel<F, T, R><<<blocks, WGT, 0, (hipStream_t)stream>>>(h->d_model, h->d_links, \
                                                 h->cfg, h->n, h->d_state, targets, nsub, net_force, applied_torque)
  if (dr) {
    if (refresh) ZB_SUB(true, true, true);
    else if (tgs) ZB_SUB(true, true, false);
    else ZB_SUB(true, false, false);
  } else {
    if (refresh) ZB_SUB(false, true, true);
    else if (tgs) ZB_SUB(false, true, false);
    else ZB_SUB(false, false, false);
  }
#undef ZB_SUB
  const int rc = launch_check("zb_substeps_kernel");
  if (rc || !h->d_wc) return rc;
  // the physics moved: the self-contact cache describes another state (cold start next step)
  zb_wc_fill_kernel<<<(h->n * ZB_WARM_ROWS + 255) / 256, 256, 0, (hipStream_t)stream>>>(h->n, h->d_wc, nullptr, h->n);
  return launch_check("zb_wc_fill_kernel");
}

int zb_pair_manifold_mode(const float* pairs, int n, float margin, int mode, float* out, void* stream) {
  if (!pairs || !out || n < 1 || mode < 1 || mode > 3) return set_err(-1, "zb_pair_manifold", hipSuccess);
  zb_manifold_kernel<<<(4 * n + 63) / 64, 64, 0, (hipStream_t)stream>>>(pairs, n, margin, mode, out);
  return launch_check("zb_manifold_kernel");
}

int zb_pair_manifold(const float* pairs, int n, float margin, float* out, void* stream) {
  return zb_pair_manifold_mode(pairs, n, margin, 2, out, stream);
}

int zb_gjk_pairs(const float* pairs, const float* v0, int n, float margin, float* out, void* stream) {
  if (!pairs || !out || n < 1) return set_err(-1, "zb_gjk_pairs", hipSuccess);
  const int threads = 4 * n;
  zb_gjk_kernel<<<(threads + 63) / 64, 64, 0, (hipStream_t)stream>>>(pairs, v0, n, margin, out);
  return launch_check("zb_gjk_kernel");
}

}  // extern "C"
