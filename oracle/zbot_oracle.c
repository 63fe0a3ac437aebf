/*
 * zbot_oracle.c — CPU ORACLE for the zbot-6b-walking-v2 hot path. TEST INFRASTRUCTURE ONLY.
 *
 * Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may load this library,
 * and only as the checker / CPU baseline. The product path (zbot_lab_amd, libzbot.so) never
 * links or calls it and fails loudly when its HIP extension is missing.
 *
 * What it restates (reference paths relative to the reference repo root):
 *   MDP  : ZbotDirectEnvV2 (source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6dof_bipedal_env_v2.py)
 *          _pre_physics_step 276-287, _get_observations 312-369, _get_rewards 371-382 and the
 *          13 reward terms 461-561, _get_dones 384-411, _reset_idx 413-459; DirectRLEnv.step
 *          order; Isaac Lab ContactSensor lazy update semantics
 *          (DESIGN.md §4). PINNED against golden vectors generated from the reference's own v2
 *          code (tests/golden/, tools/gen_mdp_goldens.py) by zbo_mdp_eval / zbo_pre_physics.
 *   Model: ZBOT_6S_CFG (source/zbot/zbot/assets/zbot_cfg.py:621-669) + zbot_6s_new.usd;
 *          forward kinematics PINNED to the reference's printed known answers (v2.py:403-404,
 *          v4.py:816) in tests/test_model.py.
 *   Physics (PhysX 5 articulation + contact; closed source, absent here): PARITY UNPINNED against
 *          PhysX. This is the simulator's own algorithm, checked only by physical
 *          invariants (free fall, momentum without contact, PD response, resting contact) and
 *          used as the reference the HIP kernel must match.
 *
 * Physics substep (same algorithm as the HIP kernel):
 *   FK of 7 composites -> world spatial inertias about P = root origin -> RNEA bias forces
 *   (gravity as base acceleration) -> CRBA mass matrix -> implicit PD drives (armature
 *   dt*kd + dt^2*kp on the joint diagonal; a joint whose implicit torque exceeds the effort
 *   limit is re-solved with an explicit +-limit torque and no armature) -> Cholesky M = L L^T ->
 *   contacts (circle-pair support points vs plane, GJK on rounded disk hulls for self collision) -> projected
 *   Gauss-Seidel on the whitened velocity w = L^T u with rows Y = L^-1 J^T (Coulomb disk
 *   friction) -> u = L^-T w -> joint speed clamp -> semi-implicit Euler, joint wrap.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/zbot.h"

#ifndef ZBO_REAL
#define ZBO_REAL float
#endif
typedef ZBO_REAL real;

#define NB ZB_NUM_BODIES
#define ND ZB_NUM_DOF
#define NL ZB_NUM_LINKS
#define NV (6 + ND)  /* generalized velocity: [omega(3), v_P(3), qdot(6)] */
#define NC_MAX ZB_MAX_CONTACTS /* contact slots per env per substep (= the HIP kernel) */
#define NCAND_PER_LINK 4
#define RIM_EPS 1e-3 /* m; = 2% of the 5 cm module radius */
/* Self collision: each link's shape (the convex hull of its two circles) is written as a core
 * hull Minkowski-summed with a ball of radius CORE_M, PhysX-PCM style: the core is the hull of the
 * two circles moved CORE_M into the shape along their plane normals with radius r - CORE_M. The
 * caps (disk faces) are exact, the rims are rounded with radius CORE_M. Pair distance = GJK
 * distance of the cores - 2 CORE_M (exact up to the rim rounding, for penetrations < 2 CORE_M). */
#define CORE_M 0.004
#define GJK_MAX_IT 16
#define GJK_TOL 1e-5 /* m: stop when the upper (|v|) and best lower (dir.w / |dir|) distance bounds are this close */
#define GJK_TILT 0.01 /* warm start: tilt of the first three support directions (rad) */
#define TWO_PI 6.283185307179586
#define PI_R 3.14159265358979323846

/* ------------------------------------------------------------------------- small math */
static inline void v3_cross(const real a[3], const real b[3], real o[3]) {
  real x = a[1] * b[2] - a[2] * b[1], y = a[2] * b[0] - a[0] * b[2], z = a[0] * b[1] - a[1] * b[0];
  o[0] = x; o[1] = y; o[2] = z;
}
static inline real v3_dot(const real a[3], const real b[3]) { return a[0] * b[0] + a[1] * b[1] + a[2] * b[2]; }
static inline void q_mul(const real a[4], const real b[4], real o[4]) {
  real w = a[0] * b[0] - a[1] * b[1] - a[2] * b[2] - a[3] * b[3];
  real x = a[0] * b[1] + a[1] * b[0] + a[2] * b[3] - a[3] * b[2];
  real y = a[0] * b[2] - a[1] * b[3] + a[2] * b[0] + a[3] * b[1];
  real z = a[0] * b[3] + a[1] * b[2] - a[2] * b[1] + a[3] * b[0];
  o[0] = w; o[1] = x; o[2] = y; o[3] = z;
}
static inline void q_to_mat(const real q[4], real R[9]) {
  real w = q[0], x = q[1], y = q[2], z = q[3];
  R[0] = 1 - 2 * (y * y + z * z); R[1] = 2 * (x * y - w * z);     R[2] = 2 * (x * z + w * y);
  R[3] = 2 * (x * y + w * z);     R[4] = 1 - 2 * (x * x + z * z); R[5] = 2 * (y * z - w * x);
  R[6] = 2 * (x * z - w * y);     R[7] = 2 * (y * z + w * x);     R[8] = 1 - 2 * (x * x + y * y);
}
static inline void m3_v(const real R[9], const real v[3], real o[3]) {
  real x = R[0] * v[0] + R[1] * v[1] + R[2] * v[2];
  real y = R[3] * v[0] + R[4] * v[1] + R[5] * v[2];
  real z = R[6] * v[0] + R[7] * v[1] + R[8] * v[2];
  o[0] = x; o[1] = y; o[2] = z;
}
static inline void q_normalize(real q[4]) {
  real n = (real)sqrt((double)(q[0] * q[0] + q[1] * q[1] + q[2] * q[2] + q[3] * q[3]));
  for (int i = 0; i < 4; ++i) q[i] /= n;
}
static inline real clampr(real x, real lo, real hi) { return x < lo ? lo : (x > hi ? hi : x); }
static inline real sqrtr(real x) { return (real)sqrt((double)x); }

/* splitmix64 finaliser: counter-based hash shared with the kernel for episode-length draws */
static inline uint64_t zb_hash64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

/* ------------------------------------------------------------------------- model (real) */
typedef struct {
  real body_mass[NB], body_com[NB][3], body_I[NB][6];
  real jp_pos[ND][3], jp_rot[ND][4], jc_pos[ND][3], jc_rot[ND][4];
  int link_body[NL];
  real link_pos[NL][3], link_rot[NL][4], link_com[NL][3];
  real circle[NL][2][9], bound[NL][4];
  real core[NL][2][9];                /* core circles of the self-collision shape (body frame) */
  int circle_dup[NL];                 /* bit ci: duplicate of a lower link's mated face (skipped) */
  int npairs, pairs[ZB_MAX_SELF_PAIRS][2];
  real root_pos0[3], root_quat0[4], jq0[ND];
  real kp, kd, effort, vlim, max_depen, wmax;
  int base_link, foot_links[2], undesired[10];
  real api_t[3], api_q[4];            /* Isaac Lab root in the chain root's frame (v09: the base) */
  int api_index[ND];                  /* chain joint j -> Isaac Lab joint order */
  real api_sign[ND];
} mdl_t;

static void load_mdl(const zb_model* m, mdl_t* o) {
  for (int b = 0; b < NB; ++b) {
    o->body_mass[b] = m->body_mass[b];
    for (int a = 0; a < 3; ++a) o->body_com[b][a] = m->body_com[b][a];
    for (int a = 0; a < 6; ++a) o->body_I[b][a] = m->body_inertia[b][a];
  }
  for (int j = 0; j < ND; ++j) {
    for (int a = 0; a < 3; ++a) { o->jp_pos[j][a] = m->joint_parent_pos[j][a]; o->jc_pos[j][a] = m->joint_child_pos[j][a]; }
    for (int a = 0; a < 4; ++a) { o->jp_rot[j][a] = m->joint_parent_rot[j][a]; o->jc_rot[j][a] = m->joint_child_rot[j][a]; }
    o->jq0[j] = m->default_joint_pos[j];
  }
  for (int l = 0; l < NL; ++l) {
    o->link_body[l] = m->link_body[l];
    o->circle_dup[l] = m->link_circle_dup[l];
    for (int a = 0; a < 3; ++a) { o->link_pos[l][a] = m->link_pos[l][a]; o->link_com[l][a] = m->link_com[l][a]; }
    for (int a = 0; a < 4; ++a) { o->link_rot[l][a] = m->link_rot[l][a]; o->bound[l][a] = m->link_bound[l][a]; }
    for (int c = 0; c < 2; ++c) {
      for (int a = 0; a < 9; ++a) o->circle[l][c][a] = m->link_circle[l][c][a];
    }
  }
  for (int l = 0; l < NL; ++l)
    for (int c = 0; c < 2; ++c) {
      const real* C = o->circle[l][c];
      const real* O = o->circle[l][1 - c];
      real n[3];
      v3_cross(C + 3, C + 6, n);
      real nn = sqrtr(v3_dot(n, n));
      real r = sqrtr(v3_dot(C + 3, C + 3));
      real to[3] = {O[0] - C[0], O[1] - C[1], O[2] - C[2]};
      real sg = v3_dot(n, to) < 0 ? (real)-1 : (real)1; /* into the shape */
      for (int a = 0; a < 3; ++a) {
        o->core[l][c][a] = C[a] + sg * (real)CORE_M * n[a] / nn;
        o->core[l][c][3 + a] = C[3 + a] * (r - (real)CORE_M) / r;
        o->core[l][c][6 + a] = C[6 + a] * (r - (real)CORE_M) / r;
      }
    }
  o->npairs = m->num_self_pairs;
  for (int p = 0; p < o->npairs; ++p) { o->pairs[p][0] = m->self_pairs[p][0]; o->pairs[p][1] = m->self_pairs[p][1]; }
  for (int a = 0; a < 3; ++a) o->root_pos0[a] = m->default_root_pos[a];
  for (int a = 0; a < 4; ++a) o->root_quat0[a] = m->default_root_quat[a];
  o->kp = m->kp; o->kd = m->kd; o->effort = m->effort_limit; o->vlim = m->velocity_limit;
  o->max_depen = m->max_depenetration_velocity;
  o->wmax = m->max_angular_velocity;
  o->base_link = m->base_link;
  o->foot_links[0] = m->foot_links[0]; o->foot_links[1] = m->foot_links[1];
  for (int k = 0; k < 10; ++k) o->undesired[k] = m->undesired_links[k];
  for (int a = 0; a < 3; ++a) o->api_t[a] = m->api_root_in_root[a];
  for (int a = 0; a < 4; ++a) o->api_q[a] = m->api_root_in_root[3 + a];
  for (int j = 0; j < ND; ++j) { o->api_index[j] = m->api_joint_index[j]; o->api_sign[j] = m->api_joint_sign[j]; }
}

/* ------------------------------------------------------------------------- per-env state */
typedef struct {
  real root_pos[3], root_quat[4], root_linvel[3], root_angvel[3];
  real jq[ND], jqd[ND];
} phys_t;

typedef struct {
  real p_delta[ND], actions[ND];
  real center_z_last;                 /* standup only (standup.py:511) */
  real mu[NL], mu_d[NL];              /* standup / manager: per-link static / dynamic friction (DR) */
  real commands[3], target_yaw, interval_left, current_yaw; /* v4 (2 commands) / manager (3; interval_left =
                                                             command time_left) */
  real cmd_standing, metrics[2];      /* manager only */
  real feet_fn_hist[3][2];            /* manager only: |net force| of the feet, per physics step */
  real feet_down_pos[2][3], feet_step_len[2], feet_f_last[2];
  real heading_sum, yerr_sum, force_sum; /* force_sum: v2 step0's feet_force_sum (v2.py:238) */
  real feet_fz_hist[ZB_HIST][2], undes_fmax_hist[ZB_HIST];
  real feet_air_cur[2], feet_air_last[2], feet_contact_cur[2], feet_contact_last[2];
  int32_t ep_len;
  real ep_sums[ZB_MAX_REWARD_TERMS];
} mdp_t;

/* persistent self-contact cache (every task): {n, code} of the first ZB_WARM_SLOTS
 * kept self contacts of the previous step's last substep, the GJK warm start of the next step's
 * first substep (code = (la << 4) + lb + 1; -1: none). Not part of the state rows: set_state and
 * resets invalidate it; zbo_{get,set}_contact_cache copy it (ZB_WARM_ROWS x N, the kernel's rows). */
typedef struct { phys_t ph; mdp_t md; float wc[ZB_WARM_ROWS]; } env_t;
static void wc_invalidate(float* wc) {
  for (int r = 0; r < ZB_WARM_ROWS; ++r) wc[r] = (r & 3) == 3 ? -1.f : 0.f;
}

struct zbo_sim {
  mdl_t m;
  zb_task_cfg c;
  int n;
  uint64_t seed, call_counter; /* zb_step / zb_reset calls so far (RNG stream position) */
  uint64_t steps;               /* common_step_counter (zb_step calls) */
  int stage;                    /* curriculum stage */
  float vel[2], yaw[2], prob_pos; /* v4 command sampling params (changed by the curricula) */
  int ring_n, ring_head;
  float ring_vel[ZB_V4_RING], ring_yaw[ZB_V4_RING];
  env_t* env;
  float log_means[ZB_LOG_LEN];
  int32_t log_counts[ZB_LOG_COUNTS];
  int changed;                  /* manager: lin_vel_cmd_levels widened the ranges in this call */
  double met_acc[2];            /* manager: summed command metrics of this call's reset envs */
  int nclose;                   /* manager: feet_close terminations of this call */
  int32_t* act;                 /* [n][2] loaded ground / self contacts summed over substeps (test hook) */
};
typedef struct zbo_sim zbo_sim;

/* ------------------------------------------------------------------------- kinematics */
typedef struct {
  real q[NB][4], R[NB][9], p[NB][3];  /* body frames; p relative to P = root origin */
  real axis[ND][3], org[ND][3];       /* joint axis (world) and point (rel P) */
} kin_t;

/* X_{b+1} = X_b * T(jp_pos, jp_rot) * Rz(q_b) * T(jc_pos, jc_rot)  (PhysX composition order) */
static void fk(const mdl_t* m, const phys_t* s, kin_t* k) {
  for (int a = 0; a < 4; ++a) k->q[0][a] = s->root_quat[a];
  q_normalize(k->q[0]);
  q_to_mat(k->q[0], k->R[0]);
  k->p[0][0] = k->p[0][1] = k->p[0][2] = 0;
  for (int j = 0; j < ND; ++j) {
    real qj[4], Rj[9], t[3];
    q_mul(k->q[j], m->jp_rot[j], qj);
    q_to_mat(qj, Rj);
    m3_v(k->R[j], m->jp_pos[j], t);
    for (int a = 0; a < 3; ++a) { k->org[j][a] = k->p[j][a] + t[a]; k->axis[j][a] = Rj[3 * a + 2]; }
    real h = (real)0.5 * s->jq[j];
    real qz[4] = {(real)cos((double)h), 0, 0, (real)sin((double)h)};
    real qa[4];
    q_mul(qj, qz, qa);
    real Ra[9];
    q_to_mat(qa, Ra);
    m3_v(Ra, m->jc_pos[j], t);
    for (int a = 0; a < 3; ++a) k->p[j + 1][a] = k->org[j][a] + t[a];
    q_mul(qa, m->jc_rot[j], k->q[j + 1]);
    q_normalize(k->q[j + 1]);
    q_to_mat(k->q[j + 1], k->R[j + 1]);
  }
}

/* link l world pose: position relative to P, quaternion */
static void link_pose(const mdl_t* m, const kin_t* k, int l, real pos[3], real quat[4]) {
  int b = m->link_body[l];
  real t[3];
  m3_v(k->R[b], m->link_pos[l], t);
  for (int a = 0; a < 3; ++a) pos[a] = k->p[b][a] + t[a];
  q_mul(k->q[b], m->link_rot[l], quat);
}

/* spatial velocity of every body at P: V = [omega; v_P] */
static void body_vel(const kin_t* k, const phys_t* s, real V[NB][6]) {
  for (int a = 0; a < 3; ++a) { V[0][a] = s->root_angvel[a]; V[0][3 + a] = s->root_linvel[a]; }
  for (int j = 0; j < ND; ++j) {
    real S[6], oxa[3];
    v3_cross(k->org[j], k->axis[j], oxa);
    for (int a = 0; a < 3; ++a) { S[a] = k->axis[j][a]; S[3 + a] = oxa[a]; }
    for (int a = 0; a < 6; ++a) V[j + 1][a] = V[j][a] + S[a] * s->jqd[j];
  }
}

/* world linear velocity of a point x (rel P) moving with body b */
static void point_vel(const real V[6], const real x[3], real o[3]) {
  real c[3];
  v3_cross(V, x, c);
  for (int a = 0; a < 3; ++a) o[a] = V[3 + a] + c[a];
}

/* ------------------------------------------------------------------------- spatial algebra */
typedef struct { real m, h[3], I[6]; } sinertia; /* about P: I = [xx yy zz xy xz yz] */

static inline void sym_mv(const real I[6], const real w[3], real o[3]) {
  real x = I[0] * w[0] + I[3] * w[1] + I[4] * w[2];
  real y = I[3] * w[0] + I[1] * w[1] + I[5] * w[2];
  real z = I[4] * w[0] + I[5] * w[1] + I[2] * w[2];
  o[0] = x; o[1] = y; o[2] = z;
}
/* f = I V : n = I w + h x v ; f = m v - h x w */
static void si_mul(const sinertia* I, const real V[6], real f[6]) {
  real Iw[3], hv[3], hw[3];
  sym_mv(I->I, V, Iw);
  v3_cross(I->h, V + 3, hv);
  v3_cross(I->h, V, hw);
  for (int a = 0; a < 3; ++a) { f[a] = Iw[a] + hv[a]; f[3 + a] = I->m * V[3 + a] - hw[a]; }
}
static void si_add(sinertia* a, const sinertia* b) {
  a->m += b->m;
  for (int i = 0; i < 3; ++i) a->h[i] += b->h[i];
  for (int i = 0; i < 6; ++i) a->I[i] += b->I[i];
}
/* motion cross: V x_m S = [w x a ; w x b + v x a] */
static void crossm(const real V[6], const real S[6], real o[6]) {
  real t1[3], t2[3], t3[3];
  v3_cross(V, S, t1);
  v3_cross(V, S + 3, t2);
  v3_cross(V + 3, S, t3);
  for (int a = 0; a < 3; ++a) { o[a] = t1[a]; o[3 + a] = t2[a] + t3[a]; }
}
/* force cross: V x_f F = [w x n + v x f ; w x f] */
static void crossf(const real V[6], const real F[6], real o[6]) {
  real t1[3], t2[3], t3[3];
  v3_cross(V, F, t1);
  v3_cross(V + 3, F + 3, t2);
  v3_cross(V, F + 3, t3);
  for (int a = 0; a < 3; ++a) { o[a] = t1[a] + t2[a]; o[3 + a] = t3[a]; }
}

/* world spatial inertia of body b about P */
static void body_sinertia(const mdl_t* m, const kin_t* k, int b, sinertia* o) {
  const real* R = k->R[b];
  real c[3];
  m3_v(R, m->body_com[b], c);
  for (int a = 0; a < 3; ++a) c[a] += k->p[b][a];
  /* Ic_world = R Ilocal R^T */
  const real* L = m->body_I[b];
  real Il[9] = {L[0], L[3], L[4], L[3], L[1], L[5], L[4], L[5], L[2]};
  real T[9], W[9];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) T[3 * i + j] = R[3 * i] * Il[j] + R[3 * i + 1] * Il[3 + j] + R[3 * i + 2] * Il[6 + j];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) W[3 * i + j] = T[3 * i] * R[3 * j] + T[3 * i + 1] * R[3 * j + 1] + T[3 * i + 2] * R[3 * j + 2];
  real mm = m->body_mass[b];
  real cc = v3_dot(c, c);
  o->m = mm;
  for (int a = 0; a < 3; ++a) o->h[a] = mm * c[a];
  o->I[0] = W[0] + mm * (cc - c[0] * c[0]);
  o->I[1] = W[4] + mm * (cc - c[1] * c[1]);
  o->I[2] = W[8] + mm * (cc - c[2] * c[2]);
  o->I[3] = W[1] - mm * c[0] * c[1];
  o->I[4] = W[2] - mm * c[0] * c[2];
  o->I[5] = W[5] - mm * c[1] * c[2];
}

/* ------------------------------------------------------------------------- contacts */
typedef struct {
  int la, lb;          /* links (lb = -1 for ground) */
  real x[3];           /* contact point, rel P */
  real n[3];           /* normal: impulse on la along +n */
  real sep;            /* separation (negative = penetration) */
  int rim;             /* ground: 4 circle + rim rotation of the candidate (ground_rim_point) */
} contact_t;

/* Candidate list (canonical order): ground candidates link by link (<= NCAND_PER_LINK each),
 * then self-collision candidates in link-pair order (one per pair: hull_pair), at most NSELF_MAX.
 * When more than NC_MAX candidates exist the NC_MAX smallest by (sep, canonical index) are kept;
 * the kept contacts are solved in canonical order. Same rule as the kernel's quad selection. */
#define NSELF_MAX 18
#define NCAND_MAX (NL * NCAND_PER_LINK + NSELF_MAX)
typedef struct { contact_t c[NCAND_MAX]; int n; } clist_t;

static void select_contacts(clist_t* L) {
  if (L->n <= NC_MAX) return;
  int keep[NCAND_MAX];
  for (int i = 0; i < L->n; ++i) {
    int rank = 0;
    for (int j = 0; j < L->n; ++j)
      if (L->c[j].sep < L->c[i].sep || (L->c[j].sep == L->c[i].sep && j < i)) ++rank;
    keep[i] = rank < NC_MAX;
  }
  int k = 0;
  for (int i = 0; i < L->n; ++i)
    if (keep[i]) L->c[k++] = L->c[i];
  L->n = k;
}

/* the persistent self-contact cache (env_t.wc) as the first substep's warm-start list, and the
 * last substep's kept self contacts, in slot order, back into it (the kernel's wc_load /
 * wc_extract) */
static void wc_warm_list(const float* wc, clist_t* wl) {
  wl->n = 0;
  for (int r = 0; r < ZB_WARM_SLOTS; ++r) {
    const int code = (int)wc[4 * r + 3];
    if (code < 1) continue;
    contact_t* c = &wl->c[wl->n++];
    c->la = code >> 4; c->lb = (code & 15) - 1;
    for (int a = 0; a < 3; ++a) c->n[a] = wc[4 * r + a];
  }
}
static void wc_invalidate(float* wc);
static void wc_store(const clist_t* wl, float* wc) {
  int r = 0;
  wc_invalidate(wc);
  for (int j = 0; j < wl->n && r < ZB_WARM_SLOTS; ++j) {
    if (wl->c[j].lb < 0) continue;
    int dup = 0; /* a manifold's points share the pair's normal: one entry per pair */
    for (int i = 0; i < j; ++i) dup |= wl->c[i].la == wl->c[j].la && wl->c[i].lb == wl->c[j].lb;
    if (dup) continue;
    for (int a = 0; a < 3; ++a) wc[4 * r + a] = (float)wl->c[j].n[a];
    wc[4 * r + 3] = (float)((wl->c[j].la << 4) + wl->c[j].lb + 1);
    ++r;
  }
}

/* ------------------------------------------------------------------ self collision (GJK)
 * World-frame core circles of link l: centre, two semi-axes (radius baked in). */
typedef struct { real c[2][9]; } hull_t;
static double g_gjk_tol = GJK_TOL;
static _Thread_local int g_gjk_last_it; /* probe: support iterations of this thread's last hull_pair */
static double g_sensor_force_scale = 1.0; /* test hook: scales the contact forces the sensors see */
/* planted contact bug (test hook, 0 = off; tests/test_fullstate_machinery.py proves that the
 * full-state parity rule flags a device carrying one): 1 = the first ground contact of every
 * substep with mu x 1.1, 2 = the first self contact's normal flipped, 3 = the penetration push-out
 * without the max_depenetration_velocity cap; rare branches (they act in the few envs that reach
 * them): 4 = the rim manifold's end points with their normal flipped, 5 = every face-manifold
 * sample 1 mm farther from the target face (its separation + 1 mm), 6 = the overlapping-core
 * separating-axis estimate without the centre-difference axis */
static int g_plant = 0;
/* per-env contact activity (test hook): the env's [loaded ground, loaded self] counters, set by the
 * step loops around each env's step */
static _Thread_local int32_t* t_act = NULL;
static int g_gjk_warm = 1;               /* warm start within a step (test hook: 0 = always cold) */
static int g_gjk_probe = 0;              /* probe: histogram of the GJK calls the kernel would make */
static long long g_gjk_hist[GJK_MAX_IT + 2];
static long long g_gjk_uhist[64];        /* probe: undecided pairs per env-substep */

static void world_hull(const mdl_t* m, const kin_t* k, int l, hull_t* h) {
  int b = m->link_body[l];
  for (int ci = 0; ci < 2; ++ci) {
    m3_v(k->R[b], m->core[l][ci], h->c[ci]);
    m3_v(k->R[b], m->core[l][ci] + 3, h->c[ci] + 3);
    m3_v(k->R[b], m->core[l][ci] + 6, h->c[ci] + 6);
    for (int a = 0; a < 3; ++a) h->c[ci][a] += k->p[b][a];
  }
}

/* support point of the hull of two circles in direction d (a circle's support is its rim point
 * along d's in-plane part; the centre when d is normal to the disk) */
static void hull_support(const hull_t* h, const real d[3], real out[3]) {
  real best = -1e30;
  for (int ci = 0; ci < 2; ++ci) {
    const real* c = h->c[ci];
    real a = v3_dot(d, c + 3), b = v3_dot(d, c + 6);
    real nr = sqrtr(a * a + b * b);
    real p[3];
    for (int q = 0; q < 3; ++q) p[q] = c[q] + (nr > (real)1e-15 ? (a * c[3 + q] + b * c[6 + q]) / nr : 0);
    real v = v3_dot(d, p);
    if (v > best) { best = v; out[0] = p[0]; out[1] = p[1]; out[2] = p[2]; }
  }
}

/* One GJK simplex step. The simplex is the newest Minkowski point a (W[0], support point PA[0])
 * plus the retained points W[1..n] (the previous step's simplex: its newest point first). Candidates are the subsets that contain a, in the order {a},
 * {a,S1}, {a,S2}, {a,S1,S2}, {a,S3}, {a,S1,S3}, {a,S2,S3}: the affine projection of the origin with
 * all barycentric weights positive, the shortest kept (a later candidate must be strictly shorter).
 * With three retained points the tetrahedron decides whether the origin is inside (overlap; a flat
 * tetrahedron - relative volume < 1e-6 - does not count). The simplex is reduced to the winner
 * (a first, then the used points in index order) and v, lam set. Returns 1 on overlap. */
static int simplex_step(real W[4][3], real PA[4][3], int* n, real lam[4], real v[3]) {
  static const int sub[7][3] = {{0, -1, -1}, {0, 1, -1}, {0, 2, -1}, {0, 1, 2}, {0, 3, -1}, {0, 1, 3}, {0, 2, 3}};
  real best = v3_dot(W[0], W[0]);
  int bi = 0;
  real bl[3] = {1, 0, 0};
  for (int c = 0; c < 3; ++c) v[c] = W[0][c];
  for (int k = 1; k < 7; ++k) {
    int m = sub[k][2] < 0 ? 2 : 3;
    if (sub[k][m - 1] > *n) continue;
    real p[3], l[3];
    if (m == 2) {
      real e[3];
      for (int c = 0; c < 3; ++c) e[c] = W[sub[k][1]][c] - W[0][c];
      real ee = v3_dot(e, e);
      if (!(ee > (real)1e-20)) continue;
      real t = -v3_dot(W[0], e) / ee;
      if (!(t > 0 && t < 1)) continue;
      for (int c = 0; c < 3; ++c) p[c] = W[0][c] + t * e[c];
      l[0] = 1 - t; l[1] = t; l[2] = 0;
    } else {
      real e1[3], e2[3];
      for (int c = 0; c < 3; ++c) { e1[c] = W[sub[k][1]][c] - W[0][c]; e2[c] = W[sub[k][2]][c] - W[0][c]; }
      real g00 = v3_dot(e1, e1), g01 = v3_dot(e1, e2), g11 = v3_dot(e2, e2);
      real r0 = -v3_dot(W[0], e1), r1 = -v3_dot(W[0], e2);
      real det = g00 * g11 - g01 * g01;
      if (!(det > (real)1e-24 * g00 * g11)) continue;
      real ts = (r0 * g11 - r1 * g01) / det, tt = (g00 * r1 - g01 * r0) / det;
      if (!(ts > 0 && tt > 0 && ts + tt < 1)) continue;
      for (int c = 0; c < 3; ++c) p[c] = W[0][c] + ts * e1[c] + tt * e2[c];
      l[0] = 1 - ts - tt; l[1] = ts; l[2] = tt;
    }
    real d2 = v3_dot(p, p);
    if (d2 < best) {
      best = d2; bi = k;
      for (int c = 0; c < 3; ++c) { v[c] = p[c]; bl[c] = l[c]; }
    }
  }
  if (*n == 3) { /* inside the tetrahedron? barycentric coordinates of the origin (Cramer) */
    real e[3][3], x12[3];
    for (int j = 0; j < 3; ++j)
      for (int c = 0; c < 3; ++c) e[j][c] = W[j + 1][c] - W[0][c];
    v3_cross(e[1], e[2], x12);
    real det = v3_dot(e[0], x12);
    real sc = sqrtr(v3_dot(e[0], e[0]) * v3_dot(e[1], e[1]) * v3_dot(e[2], e[2]));
    if (fabs((double)det) > 1e-6 * (double)sc) {
      real m0[3] = {-W[0][0], -W[0][1], -W[0][2]}, x20[3], x01[3];
      v3_cross(e[2], e[0], x20);
      v3_cross(e[0], e[1], x01);
      real b0 = v3_dot(m0, x12) / det, b1 = v3_dot(m0, x20) / det, b2 = v3_dot(m0, x01) / det;
      if (b0 > (real)1e-5 && b1 > (real)1e-5 && b2 > (real)1e-5 && b0 + b1 + b2 < 1 - (real)1e-5) return 1;
    }
  }
  int m = bi == 0 ? 1 : (sub[bi][2] < 0 ? 2 : 3);
  real NW[4][3], NP[4][3];
  for (int j = 0; j < m; ++j)
    for (int c = 0; c < 3; ++c) { NW[j][c] = W[sub[bi][j]][c]; NP[j][c] = PA[sub[bi][j]][c]; }
  for (int j = 0; j < m; ++j)
    for (int c = 0; c < 3; ++c) { W[j][c] = NW[j][c]; PA[j][c] = NP[j][c]; }
  for (int j = 0; j < 4; ++j) lam[j] = j < m ? bl[j] : 0;
  *n = m - 1;
  return 0;
}

/* extent of a hull along unit u: each circle spans c.u +- |(u.E1, u.E2)| */
static void hull_extent(const hull_t* h, const real u[3], real* lo, real* hi) {
  for (int ci = 0; ci < 2; ++ci) {
    const real* c = h->c[ci];
    real a = v3_dot(u, c + 3), b = v3_dot(u, c + 6);
    real r = sqrtr(a * a + b * b), m = v3_dot(u, c);
    if (ci == 0 || m - r < *lo) *lo = m - r;
    if (ci == 0 || m + r > *hi) *hi = m + r;
  }
}

/* Self-collision contact of one link pair: GJK distance between the two core hulls from the
 * initial direction v0 (B -> A; the kernel passes the pair's contact normal of the previous
 * substep of the same step: warm start) or, with v0 = NULL, the hull centre difference. Stops when
 * (|v|^2 - v.w) / |v| <= GJK_TOL (the distance bounds |v| and v.w / |v| agree), after GJK_MAX_IT
 * iterations, or early (no contact) once the lower bound v.w / |v| exceeds early_margin +
 * 2 CORE_M (early_margin = margin for detection). Contact: normal (pa - pb) / d from B to A,
 * separation d - 2 CORE_M, point (pa + pb) / 2. Cores that overlap (d < 1e-6): the
 * separating-axis penetration estimate (below). Returns 1 on a contact within the margin. (The
 * kernel runs the same statement on the 4 lanes of a quad:
 * gjk_quad in zbot_sim.hip.) */
static int hull_pair(const hull_t* A, const hull_t* B, real margin, real early_margin, const real* v0,
                     contact_t* out) {
  real ca[3], cb[3], v[3];
  for (int a = 0; a < 3; ++a) {
    ca[a] = (real)0.5 * (A->c[0][a] + A->c[1][a]);
    cb[a] = (real)0.5 * (B->c[0][a] + B->c[1][a]);
  }
  if (v0) { v[0] = v0[0]; v[1] = v0[1]; v[2] = v0[2]; }
  else { v[0] = ca[0] - cb[0]; v[1] = ca[1] - cb[1]; v[2] = ca[2] - cb[2]; }
  /* warm start: the first three support directions are v0 tilted by GJK_TILT toward three
   * directions 120 degrees apart, so the simplex spans a flat face at once (a support along a
   * face normal is an arbitrary rim point) */
  real td[3][3];
  if (v0) {
    const real iv = 1 / sqrtr(v3_dot(v, v)), u[3] = {v[0] * iv, v[1] * iv, v[2] * iv};
    const real ax[3] = {fabs((double)u[0]) < 0.57 ? 1 : 0, fabs((double)u[0]) >= 0.57 && fabs((double)u[1]) < 0.57 ? 1 : 0,
                        fabs((double)u[0]) >= 0.57 && fabs((double)u[1]) >= 0.57 ? 1 : 0};
    real t1[3], t2[3];
    v3_cross(u, ax, t1);
    const real it1 = 1 / sqrtr(v3_dot(t1, t1));
    for (int a = 0; a < 3; ++a) t1[a] *= it1;
    v3_cross(u, t1, t2);
    static const float tc[3] = {1.f, -0.5f, -0.5f}, ts[3] = {0.f, 0.8660254f, -0.8660254f};
    for (int k = 0; k < 3; ++k)
      for (int a = 0; a < 3; ++a) td[k][a] = u[a] + (real)GJK_TILT * ((real)tc[k] * t1[a] + (real)ts[k] * t2[a]);
  }
  real W[4][3], PA[4][3], lam[4] = {1, 0, 0, 0};
  int n = 0, overlap = 0; /* n = retained points besides the newest W[0] */
  {
    const real* d0 = v0 ? td[0] : v;
    real nd[3] = {-d0[0], -d0[1], -d0[2]}, pa[3], pb[3];
    hull_support(A, nd, pa);
    hull_support(B, d0, pb);
    for (int a = 0; a < 3; ++a) { PA[0][a] = pa[a]; W[0][a] = pa[a] - pb[a]; v[a] = W[0][a]; }
  }
  g_gjk_last_it = 0;
  const real lim = early_margin + 2 * (real)CORE_M;
  for (int it = 0; it < GJK_MAX_IT; ++it) {
    g_gjk_last_it = it + 1;
    real vv = v3_dot(v, v);
    if (vv < (real)1e-12) { overlap = 1; break; }
    const real* dir = v0 && it < 2 ? td[it + 1] : v;
    real nd[3] = {-dir[0], -dir[1], -dir[2]}, pa[3], pb[3], w[3];
    hull_support(A, nd, pa);
    hull_support(B, dir, pb);
    for (int a = 0; a < 3; ++a) w[a] = pa[a] - pb[a];
    /* any direction bounds the distance from below by its support gap dir.w / |dir|: no contact
     * once that exceeds the margin; converged when the gap along v itself is within the
     * tolerance of |v| (so the normal v / |v| is converged too) */
    const real L = v3_dot(dir, w) / sqrtr(v3_dot(dir, dir));
    if (L > lim) return 0;
    if (dir == v && sqrtr(vv) - L <= (real)g_gjk_tol) break;
    /* the simplex (the previous newest point first) is retained as W[1..n+1], w becomes W[0] */
    for (int i = n; i >= 0; --i)
      for (int a = 0; a < 3; ++a) { W[i + 1][a] = W[i][a]; PA[i + 1][a] = PA[i][a]; }
    for (int a = 0; a < 3; ++a) { W[0][a] = w[a]; PA[0][a] = pa[a]; }
    ++n;
    if (simplex_step(W, PA, &n, lam, v)) { overlap = 1; break; }
  }
  real d = sqrtr(v3_dot(v, v));
  if (overlap || d < (real)1e-6) {
    /* overlapping cores: the separating-axis estimate of the penetration over the centre
     * difference and the four circle normals -- the axis of the largest (least negative) gap,
     * oriented B -> A, is the normal, the gap the core separation (>= -true depth); the point is
     * the mean of the hull centres (the cores' deepest points along a circle normal are a whole
     * rim, so rounding would pick one) */
    real best = -1e30, nb[3] = {0, 0, 1};
    for (int ax = 0; ax < 5; ++ax) {
      real u[3];
      if (ax == 0) {
        for (int a = 0; a < 3; ++a) u[a] = ca[a] - cb[a];
      } else {
        const hull_t* H = ax <= 2 ? A : B;
        v3_cross(H->c[(ax - 1) & 1] + 3, H->c[(ax - 1) & 1] + 6, u);
      }
      real nu = sqrtr(v3_dot(u, u));
      if (nu < (real)1e-12) continue; /* coincident centres: no centre-difference axis */
      if (g_plant == 6 && ax == 0) continue; /* planted bug */
      for (int a = 0; a < 3; ++a) u[a] /= nu;
      real alo, ahi, blo, bhi;
      hull_extent(A, u, &alo, &ahi);
      hull_extent(B, u, &blo, &bhi);
      real gp = alo - bhi, gm = blo - ahi;
      real g = gp >= gm ? gp : gm;
      if (g > best) {
        best = g;
        for (int a = 0; a < 3; ++a) nb[a] = gp >= gm ? u[a] : -u[a];
      }
    }
    out->sep = (best < 0 ? best : 0) - 2 * (real)CORE_M;
    for (int a = 0; a < 3; ++a) { out->n[a] = nb[a]; out->x[a] = (real)0.5 * (ca[a] + cb[a]); }
    return out->sep < margin;
  }
  real pa[3] = {0, 0, 0};
  for (int i = 0; i <= n; ++i)
    for (int a = 0; a < 3; ++a) pa[a] += lam[i] * PA[i][a];
  out->sep = d - 2 * (real)CORE_M;
  for (int a = 0; a < 3; ++a) {
    out->n[a] = v[a] / d;
    out->x[a] = pa[a] - (real)0.5 * v[a]; /* (pa + pb) / 2 with pb = pa - v */
  }
  return out->sep < margin;
}

/* Self-contact manifold (cfg->self_manifold; PhysX PCM keeps up to 4 points per convex pair): when
 * the nearest features of the two core hulls along the pair normal n (B -> A) are both disk faces --
 * a core circle whose plane normal is within FACE_COS of the direction (A: -n, B: +n) and that
 * supports its hull along it -- the pair contributes the corners of the faces' overlap: rim points
 * of B's core face (angles from the in-plane direction toward A's face centre: all four quarter
 * points if B's disk lies inside A's, else the tip and the two rim crossings of a lens) carried
 * along +n to A's face plane, kept if the foot lies inside A's core disk and the core gap minus
 * 2 CORE_M is within the margin; then A's rim the same way toward B (along -n). The first 4 kept
 * in that order are the manifold {x = midpoint, n, sep} (a lens: B's tip, its two crossings, A's
 * tip), all along A's face normal (n = -A's outward face normal); none kept (or the faces not both
 * present): the GJK contact alone. (The kernel runs the same statement on the 4 lanes of
 * the pair's quad: face_manifold in zbot_sim.hip.) */
#define FACE_COS 0.9659258262890683 /* cos 15 deg */
#define FACE_INSET_C 0.9995500337489875 /* cos / sin of 0.03 rad: the lens crossings moved inside */
#define FACE_INSET_S 0.029995500202495664
static double g_face_cos = FACE_COS; /* test hook (zbo_set_face_cos): the parity tests move the threshold */
static int hull_face(const hull_t* H, const real d[3], real u[3]) {
  real sv[2], uu[2][3], al[2];
  for (int ci = 0; ci < 2; ++ci) {
    const real* c = H->c[ci];
    v3_cross(c + 3, c + 6, uu[ci]);
    const real iu = 1 / sqrtr(v3_dot(uu[ci], uu[ci]));
    for (int a = 0; a < 3; ++a) uu[ci][a] *= iu;
    al[ci] = v3_dot(uu[ci], d);
    const real r = sqrtr(v3_dot(c + 3, c + 3));
    const real s2 = 1 - al[ci] * al[ci];
    sv[ci] = v3_dot(c, d) + r * sqrtr(s2 > 0 ? s2 : 0);
  }
  const int f = sv[1] > sv[0] ? 1 : 0; /* the supporting circle (circle 0 on a tie) */
  if (fabs((double)al[f]) < g_face_cos) return -1;
  const real sg = al[f] < 0 ? (real)-1 : (real)1; /* oriented along d */
  for (int a = 0; a < 3; ++a) u[a] = sg * uu[f][a];
  return f;
}
static int face_manifold(const hull_t* A, const hull_t* B, const contact_t* c0, real margin, contact_t out[4]) {
  const real nA[3] = {-c0->n[0], -c0->n[1], -c0->n[2]};
  real ua[3], ub[3];
  const int fa = hull_face(A, nA, ua), fb = hull_face(B, c0->n, ub);
  if (fa < 0 || fb < 0) return 0;
  /* the manifold's normal: A's face normal (B -> A), exact for the face pair where GJK's normal of
   * two nearly parallel faces is poorly determined (PhysX clips against a reference face too) */
  const real nr[3] = {-ua[0], -ua[1], -ua[2]};
  int k = 0;
  for (int side = 0; side < 2 && k < 4; ++side) {
    /* side 0: B's rim onto A's face along +n; side 1: A's rim onto B's face along -n */
    const real* cs = side == 0 ? B->c[fb] : A->c[fa];
    const real* us = side == 0 ? ub : ua;
    const real* ct = side == 0 ? A->c[fa] : B->c[fb];
    const real* ut = side == 0 ? ua : ub;
    const real sg = side == 0 ? (real)1 : (real)-1;
    const real rs = sqrtr(v3_dot(cs + 3, cs + 3)), rt = sqrtr(v3_dot(ct + 3, ct + 3));
    /* rim angles: measured from d0, the in-plane direction toward the other face's centre at
     * in-plane distance d. This rim inside the other disk: 0 / 90 / 180 / 270 deg; the other disk
     * inside this one: none; a lens: the tip (0) and the two rim crossings (+-alpha) moved
     * FACE_INSET rad toward the tip; apart: the tip only. Samples as (cos, sin) pairs. */
    real d0[3], d1[3];
    for (int a = 0; a < 3; ++a) d0[a] = ct[a] - cs[a];
    const real du = v3_dot(d0, us);
    for (int a = 0; a < 3; ++a) d0[a] -= du * us[a];
    const real d = sqrtr(v3_dot(d0, d0));
    if (d < (real)1e-9) { /* concentric faces: a fixed in-plane axis */
      const real ax[3] = {fabs((double)us[0]) < 0.9 ? 1 : 0, fabs((double)us[0]) < 0.9 ? 0 : 1, 0};
      const real au = v3_dot(ax, us);
      for (int a = 0; a < 3; ++a) d0[a] = ax[a] - au * us[a];
      const real id0 = 1 / sqrtr(v3_dot(d0, d0));
      for (int a = 0; a < 3; ++a) d0[a] *= id0;
    } else {
      for (int a = 0; a < 3; ++a) d0[a] /= d;
    }
    v3_cross(us, d0, d1);
    real cs_[4], sn_[4];
    int na = 0;
    if (d + rs <= rt) {
      cs_[0] = 1; sn_[0] = 0; cs_[1] = 0; sn_[1] = 1; cs_[2] = -1; sn_[2] = 0; cs_[3] = 0; sn_[3] = -1; na = 4;
    } else if (d + rt > rs) {
      cs_[0] = 1; sn_[0] = 0; na = 1;
      if (d < rs + rt) {
        const real ca = clampr((d * d + rs * rs - rt * rt) / (2 * d * rs), -1, 1);
        const real sa = sqrtr(1 - ca * ca);
        const real ci = (real)FACE_INSET_C, si = (real)FACE_INSET_S; /* rotate by -FACE_INSET */
        cs_[1] = ca * ci + sa * si; sn_[1] = sa * ci - ca * si;
        cs_[2] = cs_[1]; sn_[2] = -sn_[1];
        na = 3;
      }
    }
    const real den = sg * v3_dot(nr, ut);
    if (fabs((double)den) < 1e-6) continue;
    for (int r = 0; r < na && k < 4; ++r) {
      const real cr = cs_[r], sr = sn_[r];
      real p[3], q[3], w[3];
      for (int a = 0; a < 3; ++a) p[a] = cs[a] + rs * (cr * d0[a] + sr * d1[a]);
      for (int a = 0; a < 3; ++a) w[a] = ct[a] - p[a];
      const real t = v3_dot(w, ut) / den + (g_plant == 5 ? (real)1e-3 : 0); /* p + t sg n lies on the target face plane (planted bug 5: + 1 mm) */
      for (int a = 0; a < 3; ++a) q[a] = p[a] + t * sg * nr[a] - ct[a];
      if (v3_dot(q, q) > rt * rt) continue;
      const real sep = t - 2 * (real)CORE_M;
      if (!(sep < margin)) continue;
      contact_t* o = &out[k++];
      o->la = c0->la; o->lb = c0->lb; o->sep = sep;
      for (int a = 0; a < 3; ++a) { o->n[a] = nr[a]; o->x[a] = p[a] + (real)0.5 * t * sg * nr[a]; }
    }
  }
  return k;
}

/* Rim (ruling) manifold (cfg->self_manifold 2, round 4; PhysX PCM keeps up to 4 points per convex
 * pair): two links lying side by side touch along a line -- the nearest features are a ruling of each
 * core hull, the segment between the support points of its two circles along the pair direction (A:
 * -n, B: +n). When both rulings lie within RIM_DEG of the contact plane and of each other, the pair
 * contributes up to 3 points: the GJK point (with its GJK normal, which also warm-starts the pair's
 * GJK in the next substep), then the two ends of the rulings' overlap along A's ruling (kept when
 * more than 1 mm from the GJK point along it and within the margin), each with the normal n made
 * perpendicular to A's ruling (the component of a line contact's GJK normal along the line is
 * determined only to GJK's tolerance cone); an end's separation is the gap between the two rulings
 * along that normal at that end, minus 2 CORE_M. Rulings absent or crossing: the GJK
 * contact alone. (The kernel: the rim branch of quad_manifold, on the pair's quad.) */
#define RIM_COS 0.9961946980917455 /* cos 5 deg */
static double g_rim_cos = RIM_COS; /* moved with the face threshold by zbo_set_face_cos (15 deg -> 5 deg scale) */
static void hull_ruling(const hull_t* H, const real d[3], real p[2][3]) {
  for (int ci = 0; ci < 2; ++ci) {
    const real* c = H->c[ci];
    const real a = v3_dot(d, c + 3), b = v3_dot(d, c + 6);
    const real nr = sqrtr(a * a + b * b);
    for (int q = 0; q < 3; ++q) p[ci][q] = c[q] + (nr > (real)1e-15 ? (a * c[3 + q] + b * c[6 + q]) / nr : 0);
  }
}
static int rim_manifold(const hull_t* A, const hull_t* B, const contact_t* c0, real margin, contact_t out[3]) {
  const real* n = c0->n;
  const real nA[3] = {-n[0], -n[1], -n[2]};
  real pa[2][3], pb[2][3];
  hull_ruling(A, nA, pa);
  hull_ruling(B, n, pb);
  real sa[3], sb[3];
  for (int q = 0; q < 3; ++q) { sa[q] = pa[1][q] - pa[0][q]; sb[q] = pb[1][q] - pb[0][q]; }
  const real la = sqrtr(v3_dot(sa, sa)), lb = sqrtr(v3_dot(sb, sb));
  if (la < (real)1e-3 || lb < (real)1e-3) return 0;
  const real sin_t = (real)sqrt(1.0 - g_rim_cos * g_rim_cos);
  /* both rulings within RIM_DEG of the contact plane, and of each other */
  if (fabs((double)v3_dot(sa, n)) > sin_t * la || fabs((double)v3_dot(sb, n)) > sin_t * lb) return 0;
  if (fabs((double)v3_dot(sa, sb)) < g_rim_cos * la * lb) return 0;
  real ah[3];
  for (int q = 0; q < 3; ++q) ah[q] = sa[q] / la;
  real nr[3];
  const real na = v3_dot(n, ah);
  for (int q = 0; q < 3; ++q) nr[q] = n[q] - na * ah[q];
  const real inr = 1 / sqrtr(v3_dot(nr, nr));
  for (int q = 0; q < 3; ++q) nr[q] *= inr;
  /* the overlap of the rulings along A's: t in [0, la] on A, B's ends at tb0, tb1 */
  real w0[3], w1[3], wg[3];
  for (int q = 0; q < 3; ++q) { w0[q] = pb[0][q] - pa[0][q]; w1[q] = pb[1][q] - pa[0][q]; wg[q] = c0->x[q] - pa[0][q]; }
  const real tb0 = v3_dot(w0, ah), tb1 = v3_dot(w1, ah), tg = v3_dot(wg, ah);
  const real lo = fmax((double)0, (double)(tb0 < tb1 ? tb0 : tb1)), hi = fmin((double)la, (double)(tb0 < tb1 ? tb1 : tb0));
  int k = 0;
  out[k++] = *c0; /* (its own GJK normal: the pair's warm start in the next substep, as without a rim) */
  if (!(hi - lo > (real)1e-3)) return k;
  const real dtb = tb1 - tb0;
  for (int e = 0; e < 2; ++e) {
    const real t = e == 0 ? lo : hi;
    if (!(fabs((double)(t - tg)) > 1e-3)) continue;
    const real ua = t / la, ub = (t - tb0) / dtb;
    real xa[3], xb[3], g[3];
    for (int q = 0; q < 3; ++q) {
      xa[q] = pa[0][q] + ua * sa[q];
      xb[q] = pb[0][q] + ub * sb[q];
      g[q] = xa[q] - xb[q];
    }
    const real sep = v3_dot(g, nr) - 2 * (real)CORE_M;
    if (!(sep < margin)) continue;
    contact_t* o = &out[k++];
    o->la = c0->la; o->lb = c0->lb; o->sep = sep; o->rim = -1;
    const real fl = g_plant == 4 ? (real)-1 : (real)1; /* planted bug 4: the end's normal flipped */
    for (int q = 0; q < 3; ++q) { o->n[q] = fl * nr[q]; o->x[q] = (real)0.5 * (xa[q] + xb[q]); }
  }
  return k;
}
/* Ruling on a face (cfg->self_manifold 3, round 5; PhysX PCM keeps up to 4 points per convex pair):
 * one hull presents a face along the pair direction (hull_face: a core circle within FACE_COS of it
 * that supports the hull) and the other a ruling (hull_ruling) within RIM_DEG of the contact plane --
 * a link lying on another's cap. Up to 3 points: the GJK point (its GJK normal: the pair's warm
 * start), then the two ends of the ruling's stretch over the face's core disk (the segment clipped
 * to the disk in the face plane), kept when more than 1 mm from the GJK point along the ruling and
 * within the margin, each with the face's exact normal (B -> A) and the ruling end's distance to the
 * face plane minus 2 CORE_M, at the midpoint between the end and its foot on the face. */
static int rim_face_manifold(const hull_t* A, const hull_t* B, const contact_t* c0, real margin, contact_t out[3]) {
  const real* n = c0->n;
  const real nA[3] = {-n[0], -n[1], -n[2]};
  real ua[3], ub[3], pr[2][3];
  const int fa = hull_face(A, nA, ua), fb = hull_face(B, n, ub);
  if ((fa >= 0) == (fb >= 0)) return 0;
  /* the face (centre cf, outward normal uf toward the other hull, core radius rf) and the ruling */
  const real* cf = fa >= 0 ? A->c[fa] : B->c[fb];
  const real* uf = fa >= 0 ? ua : ub;
  if (fa >= 0) hull_ruling(B, n, pr);
  else hull_ruling(A, nA, pr);
  real nr[3];  /* the contact normal B -> A: -A's face normal, or B's */
  for (int q = 0; q < 3; ++q) nr[q] = fa >= 0 ? -uf[q] : uf[q];
  real sv[3];
  for (int q = 0; q < 3; ++q) sv[q] = pr[1][q] - pr[0][q];
  const real ls = sqrtr(v3_dot(sv, sv));
  if (ls < (real)1e-3) return 0;
  const real sin_t = (real)sqrt(1.0 - g_rim_cos * g_rim_cos);
  if (fabs((double)v3_dot(sv, n)) > sin_t * ls) return 0;
  /* the stretch of the ruling whose foot lies inside the face's core disk: |P (x(t) - cf)| <= rf */
  const real rf = sqrtr(v3_dot(cf + 3, cf + 3));
  real q0[3], qs[3];
  for (int q = 0; q < 3; ++q) q0[q] = pr[0][q] - cf[q];
  const real q0u = v3_dot(q0, uf), qsu = v3_dot(sv, uf);
  for (int q = 0; q < 3; ++q) { q0[q] -= q0u * uf[q]; qs[q] = sv[q] - qsu * uf[q]; }
  const real a = v3_dot(qs, qs), b = 2 * v3_dot(q0, qs), c = v3_dot(q0, q0) - rf * rf;
  const real disc = b * b - 4 * a * c;
  int k = 0;
  out[k++] = *c0;
  if (!(a > (real)1e-12) || !(disc > 0)) return k;
  const real sq = sqrtr(disc);
  const real lo = fmax(0.0, (double)((-b - sq) / (2 * a))), hi = fmin(1.0, (double)((-b + sq) / (2 * a)));
  if (!((hi - lo) * ls > (real)1e-3)) return k;
  real wg[3];
  for (int q = 0; q < 3; ++q) wg[q] = c0->x[q] - pr[0][q];
  const real tg = v3_dot(wg, sv) / (ls * ls);
  for (int e = 0; e < 2; ++e) {
    const real t = e == 0 ? lo : hi;
    if (!(fabs((double)(t - tg)) * ls > 1e-3)) continue;
    real x[3], g;
    for (int q = 0; q < 3; ++q) x[q] = pr[0][q] + t * sv[q];
    {
      real d[3];
      for (int q = 0; q < 3; ++q) d[q] = x[q] - cf[q];
      g = v3_dot(d, uf);
    }
    const real sep = g - 2 * (real)CORE_M;
    if (!(sep < margin)) continue;
    contact_t* o = &out[k++];
    o->la = c0->la; o->lb = c0->lb; o->sep = sep; o->rim = -1;
    for (int q = 0; q < 3; ++q) { o->n[q] = nr[q]; o->x[q] = x[q] - (real)0.5 * g * uf[q]; }
  }
  return k;
}

/* the self-contact manifold of cfg->self_manifold (1: faces; 2: faces, else side-by-side rims; 3:
 * faces, else a ruling on a face with at least one end point, else side-by-side rims; 0: none) */
static int self_manifold(int mode, const hull_t* A, const hull_t* B, const contact_t* c0, real margin, contact_t out[4]) {
  if (mode < 1 || !(c0->sep > -2 * (real)CORE_M + (real)1e-7)) return 0;
  int k = face_manifold(A, B, c0, margin, out);
  if (k > 0 || mode < 2) return k;
  /* (a ruling-on-face pair that keeps only its GJK point may still lie side by side: ADVICE r5) */
  if (mode >= 3 && (k = rim_face_manifold(A, B, c0, margin, out)) >= 2) return k;
  return rim_manifold(A, B, c0, margin, out);
}

/* GJK stopping tolerance (test hook: the parity tests re-run the oracle at other tolerances to tell
 * an env whose result depends on where GJK stops - an algorithmic discontinuity like the contact
 * margin - from a real mismatch) */
/* contact forces as the sensors see them scaled by s (test hook, 1 = off): the parity tests re-run
 * the oracle with the forces moved by their comparison tolerance, so that an env whose outcome
 * flips at a sensor force threshold (touchdown 10 N, is_contact 1 N, ...) within that tolerance
 * is told from a real mismatch; the physics is unaffected */
int zbo_set_sensor_force_scale(double s) {
  g_sensor_force_scale = s > 0 ? s : 1.0;
  return 0;
}

int zbo_set_plant(int mode) {
  g_plant = mode;
  return 0;
}

/* the face-alignment threshold of the self-contact manifold (test hook; 0 = the default): where a
 * pair switches between one point and a face manifold is a discontinuity like the contact margin */
int zbo_set_face_cos(double c) {
  g_face_cos = c > 0 ? c : FACE_COS;
  g_rim_cos = c > 0 ? cos(acos(c) / 3.0) : RIM_COS; /* the rim threshold moves with it (15 -> 5 deg) */
  return 0;
}

int zbo_set_gjk_tol(double tol) {
  g_gjk_tol = tol > 0 ? tol : GJK_TOL;
  return 0;
}

/* largest separating-axis gap over the centre difference and the four circle normals (the kernel's
 * hulls_separated test) */
static real sat_gap(const hull_t* A, const hull_t* B) {
  real best = -1e30;
  for (int ax = 0; ax < 5; ++ax) {
    real u[3];
    if (ax == 0) {
      for (int a = 0; a < 3; ++a) u[a] = (real)0.5 * (A->c[0][a] + A->c[1][a]) - (real)0.5 * (B->c[0][a] + B->c[1][a]);
    } else {
      const hull_t* H = ax <= 2 ? A : B;
      v3_cross(H->c[(ax - 1) & 1] + 3, H->c[(ax - 1) & 1] + 6, u);
    }
    real nu = sqrtr(v3_dot(u, u));
    if (nu < (real)1e-15) nu = (real)1e-15;
    for (int a = 0; a < 3; ++a) u[a] /= nu;
    real alo, ahi, blo, bhi;
    hull_extent(A, u, &alo, &ahi);
    hull_extent(B, u, &blo, &bhi);
    real gp = alo - bhi, gm = blo - ahi, g = gp > gm ? gp : gm;
    if (g > best) best = g;
  }
  return best;
}

/* GJK probe (test / tooling hook): the link pairs of every env that the kernel's separating-axis
 * test leaves to GJK (largest gap <= margin + 2 CORE_M), written as {env, pair, A[2][9], B[2][9]}
 * (38 floats each, at most max); returns the number of such pairs. */
int zbo_undecided_pairs(zbo_sim* s, float* out, int max) {
  int cnt = 0;
  const real lim = s->c.contact_margin + 2 * (real)CORE_M;
  for (int e = 0; e < s->n; ++e) {
    kin_t k;
    fk(&s->m, &s->env[e].ph, &k);
    for (int p = 0; p < s->m.npairs; ++p) {
      hull_t A, B;
      world_hull(&s->m, &k, s->m.pairs[p][0], &A);
      world_hull(&s->m, &k, s->m.pairs[p][1], &B);
      if (sat_gap(&A, &B) > lim) continue;
      if (cnt < max) {
        float* o = out + 38 * cnt;
        o[0] = (float)e; o[1] = (float)p;
        for (int ci = 0; ci < 2; ++ci)
          for (int q = 0; q < 9; ++q) { o[2 + 9 * ci + q] = (float)A.c[ci][q]; o[20 + 9 * ci + q] = (float)B.c[ci][q]; }
      }
      ++cnt;
    }
  }
  return cnt;
}

/* GJK tail probe (tooling, tools/gjk/tail_classes.py): the probe's GJK calls by the configuration
 * they converge to (0 no contact within the margin, 1 face on face, 2 a ruling lying on a face
 * within RIM_DEG, 3 side-by-side rulings within RIM_DEG -- the rim manifold's case --, 4 side by side
 * within FACE_DEG, 5 any other: point-like) x support iterations */
#define GJK_NCLS 6
static long long g_gjk_cls[GJK_NCLS][GJK_MAX_IT + 2];
static int gjk_class(const hull_t* A, const hull_t* B, const contact_t* c, int hit) {
  if (!hit) return 0;
  const real nA[3] = {-c->n[0], -c->n[1], -c->n[2]};
  real ua[3], ub[3];
  const int fa = hull_face(A, nA, ua), fb = hull_face(B, c->n, ub);
  if (fa >= 0 && fb >= 0) return 1;
  real pa[2][3], pb[2][3], sa[3], sb[3];
  hull_ruling(A, nA, pa);
  hull_ruling(B, c->n, pb);
  for (int q = 0; q < 3; ++q) { sa[q] = pa[1][q] - pa[0][q]; sb[q] = pb[1][q] - pb[0][q]; }
  const real la = sqrtr(v3_dot(sa, sa)), lb = sqrtr(v3_dot(sb, sb));
  const real s5 = (real)0.08715574274765817, s15 = (real)0.25881904510252074;
  const int ra5 = la > (real)1e-3 && fabs((double)v3_dot(sa, c->n)) <= s5 * la;
  const int rb5 = lb > (real)1e-3 && fabs((double)v3_dot(sb, c->n)) <= s5 * lb;
  if ((fa >= 0 && rb5) || (fb >= 0 && ra5)) return 2;
  const int ra15 = la > (real)1e-3 && fabs((double)v3_dot(sa, c->n)) <= s15 * la;
  const int rb15 = lb > (real)1e-3 && fabs((double)v3_dot(sb, c->n)) <= s15 * lb;
  const real cab = la > 0 && lb > 0 ? fabs((double)v3_dot(sa, sb)) / (la * lb) : 0;
  if (ra5 && rb5 && cab >= (real)RIM_COS) return 3;
  if (ra15 && rb15 && cab >= (real)FACE_COS) return 4;
  return 5;
}
int zbo_gjk_classes(long long* out) {
  for (int k = 0; k < GJK_NCLS; ++k)
    for (int i = 0; i < GJK_MAX_IT + 2; ++i) { out[k * (GJK_MAX_IT + 2) + i] = g_gjk_cls[k][i]; g_gjk_cls[k][i] = 0; }
  return GJK_MAX_IT + 2;
}

/* GJK probe / warm-start switches (tooling hooks): warm = 0 runs every GJK cold from the best
 * separating axis; probe = 1 histograms the support iterations of the GJK calls the kernel would
 * make (pairs the separating-axis test leaves undecided). hist: GJK_MAX_IT + 2 counters. */
int zbo_gjk_hooks(int warm, int probe, long long* hist) {
  if (warm >= 0) g_gjk_warm = warm & 1;
  if (probe >= 0) g_gjk_probe = probe;
  if (hist) {
    for (int i = 0; i < GJK_MAX_IT + 2; ++i) { hist[i] = g_gjk_hist[i]; g_gjk_hist[i] = 0; }
    for (int i = 0; i < 64; ++i) { hist[GJK_MAX_IT + 2 + i] = g_gjk_uhist[i]; g_gjk_uhist[i] = 0; }
  }
  return 0;
}

/* test entry points: hull_pair on two world-frame core hulls given as [2][9] floats (centre, two
 * semi-axes per circle) from the start direction v0 (NULL: the hull centre difference);
 * out = {contact, sep, n[3], x[3]}; returns the support iterations (tests/test_oracle_selfcollision.py,
 * tests/test_gpu_selfcollision.py, tools/gjk/probe.py) */
int zbo_hull_pair_from(const float* a, const float* b, float margin, const float* v0, float* out) {
  hull_t A, B;
  for (int ci = 0; ci < 2; ++ci)
    for (int q = 0; q < 9; ++q) { A.c[ci][q] = a[9 * ci + q]; B.c[ci][q] = b[9 * ci + q]; }
  contact_t c;
  memset(&c, 0, sizeof(c));
  real w0[3];
  if (v0) { w0[0] = v0[0]; w0[1] = v0[1]; w0[2] = v0[2]; }
  int hit = hull_pair(&A, &B, (real)margin, (real)margin, v0 ? w0 : NULL, &c);
  out[0] = (float)hit;
  out[1] = (float)c.sep;
  for (int q = 0; q < 3; ++q) { out[2 + q] = (float)c.n[q]; out[5 + q] = (float)c.x[q]; }
  return g_gjk_last_it; /* support iterations (GJK probe) */
}
/* test entry: hull_pair + the self-contact manifold (mode zbo_set_pair_manifold_mode, default 2) on
 * two world-frame core hulls; out [4][7] = {sep, n[3], x[3]} per point; returns the number of points
 * (0: no contact, 1: the GJK contact alone) */
static int g_pair_manifold_mode = 2;
int zbo_set_pair_manifold_mode(int m) {
  g_pair_manifold_mode = m;
  return 0;
}
int zbo_pair_manifold(const float* a, const float* b, float margin, float* out) {
  hull_t A, B;
  for (int ci = 0; ci < 2; ++ci)
    for (int q = 0; q < 9; ++q) { A.c[ci][q] = a[9 * ci + q]; B.c[ci][q] = b[9 * ci + q]; }
  contact_t c, mf[4];
  memset(&c, 0, sizeof(c));
  if (!hull_pair(&A, &B, (real)margin, (real)margin, NULL, &c)) return 0;
  int k = self_manifold(g_pair_manifold_mode, &A, &B, &c, (real)margin, mf);
  if (k == 0) { mf[0] = c; k = 1; }
  for (int j = 0; j < k; ++j) {
    out[7 * j] = (float)mf[j].sep;
    for (int q = 0; q < 3; ++q) { out[7 * j + 1 + q] = (float)mf[j].n[q]; out[7 * j + 4 + q] = (float)mf[j].x[q]; }
  }
  return k;
}
/* the same with the manifold mode (mirror of the library's zb_pair_manifold_mode) */
int zbo_pair_manifold_mode(const float* a, const float* b, float margin, int mode, float* out) {
  const int m0 = g_pair_manifold_mode;
  g_pair_manifold_mode = mode;
  const int k = zbo_pair_manifold(a, b, margin, out);
  g_pair_manifold_mode = m0;
  return k;
}
int zbo_hull_pair(const float* a, const float* b, float margin, float* out) {
  return zbo_hull_pair_from(a, b, margin, NULL, out);
}
/* mirror of the library's test entry zb_gjk_pairs (host pointers): pairs [n][2][2][9], v0 [n][3] or
 * NULL, out [n][9] = {contact, sep, n[3], x[3], iterations} */
int zbo_gjk_pairs(const float* pairs, const float* v0, int n, float margin, float* out, void* stream) {
  (void)stream;
  for (int k = 0; k < n; ++k)
    out[9 * k + 8] = (float)zbo_hull_pair_from(pairs + 36 * k, pairs + 36 * k + 18, margin, v0 ? v0 + 3 * k : NULL,
                                               out + 9 * k);
  return 0;
}

/* Ground: each link's shape is the convex hull of two circles (C, E1, E2 in body frame). The
 * lowest rim point of each circle plus its three 90-degree rotations along the rim are the
 * candidates (4 per circle: a flat disk resting on the plane yields a 4-point manifold);
 * per link the first NCAND_PER_LINK below the speculative margin are kept. Self: the GJK contact
 * of every non-adjacent link pair (hull_pair; the kernel's broadphase is conservative, so testing
 * all pairs here finds the same candidates). */
/* ground candidate r (0: the lowest rim point, 1-3: its 90-degree rotations along the rim) of
 * circle ci of link l at the pose k: the rim angle of the lowest point is biased by RIM_EPS toward
 * E1 so that a (nearly) flat disk gets a fixed, body-attached 4-point manifold instead of a
 * rounding-noise direction. Position relative to k's origin. */
static void ground_rim_point(const mdl_t* m, const kin_t* k, int l, int ci, int r, real x[3]) {
  const int b = m->link_body[l];
  const real* R = k->R[b];
  const real* cd = m->circle[l][ci];
  real C[3], E1[3], E2[3];
  m3_v(R, cd, C);
  m3_v(R, cd + 3, E1);
  m3_v(R, cd + 6, E2);
  for (int a = 0; a < 3; ++a) C[a] += k->p[b][a];
  real al = -E1[2] + (real)RIM_EPS, be = -E2[2];
  real nrm = sqrtr(al * al + be * be);
  real cs = 1, sn = 0;
  if (nrm > (real)1e-12) { cs = al / nrm; sn = be / nrm; }
  real cr, sr;
  if (r == 0) { cr = cs; sr = sn; }
  else if (r == 1) { cr = -sn; sr = cs; }
  else if (r == 2) { cr = -cs; sr = -sn; }
  else { cr = sn; sr = -cs; }
  for (int a = 0; a < 3; ++a) x[a] = C[a] + cr * E1[a] + sr * E2[a];
}

static void detect(const mdl_t* m, const zb_task_cfg* cfg, const kin_t* k, real Pz, const clist_t* warm,
                   clist_t* L) {
  L->n = 0;
  const real margin = cfg->contact_margin;
  for (int l = 0; l < NL; ++l) {
    const real* R = k->R[m->link_body[l]];
    /* cull: bounding sphere entirely above the margin */
    real bc[3];
    m3_v(R, m->bound[l], bc);
    if (Pz + k->p[m->link_body[l]][2] + bc[2] - m->bound[l][3] > margin) continue;
    int taken = 0;
    for (int ci = 0; ci < 2; ++ci) {
      if ((m->circle_dup[l] >> ci) & 1) continue; /* mated face: the lower link's candidates stand */
      for (int r = 0; r < 4; ++r) {
        contact_t c;
        ground_rim_point(m, k, l, ci, r, c.x);
        c.sep = Pz + c.x[2];
        c.rim = 4 * ci + r;
        /* the first NCAND_PER_LINK valid candidates in the fixed order (circle 0: lowest, +90,
         * +180, +270 degrees; then circle 1): a fixed order (not a depth sort) keeps the
         * Gauss-Seidel row order independent of rounding when rim points sit at one depth */
        if (c.sep < margin && taken < NCAND_PER_LINK) {
          c.la = l; c.lb = -1;
          c.n[0] = 0; c.n[1] = 0; c.n[2] = 1;
          L->c[L->n++] = c;
          ++taken;
        }
      }
    }
  }
  if (cfg->enable_self_collision) {
    int nself = 0, nund = 0;
    for (int p = 0; p < m->npairs && nself < NSELF_MAX; ++p) {
      int la = m->pairs[p][0], lb = m->pairs[p][1];
      hull_t A, B;
      world_hull(m, k, la, &A);
      world_hull(m, k, lb, &B);
      /* warm start: the pair's contact normal of the previous substep of this step, if kept */
      const real* v0 = NULL;
      if (warm)
        for (int j = 0; j < warm->n; ++j)
          if (warm->c[j].la == la && warm->c[j].lb == lb) { v0 = warm->c[j].n; break; }
      if (g_gjk_probe && sat_gap(&A, &B) > margin + 2 * (real)CORE_M) continue; /* kernel: no GJK */
      ++nund;
      contact_t c;
      const int hit = hull_pair(&A, &B, margin, margin, g_gjk_warm ? v0 : NULL, &c);
      if (g_gjk_probe) {
        __atomic_fetch_add(&g_gjk_hist[g_gjk_last_it], 1, __ATOMIC_RELAXED);
        __atomic_fetch_add(&g_gjk_cls[gjk_class(&A, &B, &c, hit)][g_gjk_last_it], 1, __ATOMIC_RELAXED);
      }
      if (hit) {
        c.la = la; c.lb = lb; c.rim = -1;
        contact_t mf[4];
        const int k = self_manifold(cfg->self_manifold, &A, &B, &c, margin, mf);
        if (k == 0) {
          L->c[L->n++] = c;
          ++nself;
        }
        for (int j = 0; j < k && nself < NSELF_MAX; ++j) {
          L->c[L->n++] = mf[j];
          ++nself;
        }
      }
    }
    if (g_gjk_probe) __atomic_fetch_add(&g_gjk_uhist[nund < 63 ? nund : 63], 1, __ATOMIC_RELAXED);
  }
  select_contacts(L);
}

/* tangent basis for normal n (deterministic, shared with the kernel) */
static void tangents(const real n[3], real t1[3], real t2[3]) {
  if (fabs((double)n[2]) < (real)0.9) { /* t1 = normalize(z x n) */
    real v[3] = {-n[1], n[0], 0};
    real s = sqrtr(v[0] * v[0] + v[1] * v[1]);
    t1[0] = v[0] / s; t1[1] = v[1] / s; t1[2] = 0;
  } else { /* t1 = normalize(n x x) ... = (0, n2, -n1)/|.| */
    real v[3] = {0, n[2], -n[1]};
    real s = sqrtr(v[1] * v[1] + v[2] * v[2]);
    t1[0] = 0; t1[1] = v[1] / s; t1[2] = v[2] / s;
  }
  v3_cross(n, t1, t2);
}

/* J row (length NV) of direction d at point x on body b: [x x d ; d ; S_k . f for k < b] */
static void jac_row(const kin_t* k, int b, const real x[3], const real d[3], real J[NV]) {
  real f[6];
  v3_cross(x, d, f);
  for (int a = 0; a < 3; ++a) f[3 + a] = d[a];
  for (int a = 0; a < 6; ++a) J[a] = f[a];
  for (int j = 0; j < ND; ++j) {
    if (j < b) {
      real xo[3] = {x[0] - k->org[j][0], x[1] - k->org[j][1], x[2] - k->org[j][2]};
      real c[3];
      v3_cross(xo, d, c);
      J[6 + j] = v3_dot(k->axis[j], c);
    } else {
      J[6 + j] = 0;
    }
  }
}

/* ------------------------------------------------------------------------- dense solve */
/* L L^T = A (A symmetric NVxNV, lower triangle used) */
static void cholesky(real A[NV][NV], real L[NV][NV]) {
  for (int j = 0; j < NV; ++j) {
    real s = A[j][j];
    for (int k = 0; k < j; ++k) s -= L[j][k] * L[j][k];
    real d = sqrtr(s > (real)1e-12 ? s : (real)1e-12);
    L[j][j] = d;
    real inv = (real)1 / d;
    for (int i = j + 1; i < NV; ++i) {
      real t = A[i][j];
      for (int k = 0; k < j; ++k) t -= L[i][k] * L[j][k];
      L[i][j] = t * inv;
    }
    for (int i = 0; i < j; ++i) L[i][j] = 0;
  }
}
static void fwd_sub(real L[NV][NV], const real b[NV], real y[NV]) { /* L y = b */
  for (int i = 0; i < NV; ++i) {
    real t = b[i];
    for (int k = 0; k < i; ++k) t -= L[i][k] * y[k];
    y[i] = t / L[i][i];
  }
}
static void bwd_sub(real L[NV][NV], const real y[NV], real x[NV]) { /* L^T x = y */
  for (int i = NV - 1; i >= 0; --i) {
    real t = y[i];
    for (int k = i + 1; k < NV; ++k) t -= L[k][i] * x[k];
    x[i] = t / L[i][i];
  }
}
static void lt_mul(real L[NV][NV], const real u[NV], real w[NV]) { /* w = L^T u */
  for (int i = 0; i < NV; ++i) {
    real t = 0;
    for (int k = i; k < NV; ++k) t += L[k][i] * u[k];
    w[i] = t;
  }
}

/* ------------------------------------------------------------------------- one substep */
typedef struct {
  real net_force[NL][3];   /* net contact force per link (N) of this substep */
  real applied_torque[ND]; /* Isaac Lab ImplicitActuator estimate at substep start */
} substep_out_t;

/* contact bias velocity: a speculative contact (sep >= 0) may close its gap within the step h it
 * is solved for (PGS: the substep dt; TGS: the sub-iteration dt / iterations); a penetration is
 * pushed out at baumgarte * depth per substep, capped at max_depenetration_velocity
 * (zbot_cfg.py:633) */
static real contact_bias(const zb_task_cfg* cfg, const mdl_t* m, real sep, real h, real dt) {
  if (sep >= 0) return -sep / h;
  real push = cfg->baumgarte * (-sep) / dt;
  if (g_plant == 3) return push; /* planted bug: no cap */
  return push < m->max_depen ? push : m->max_depen;
}
static void clamp_speeds(const mdl_t* m, real u[NV]) {
  for (int j = 0; j < ND; ++j) u[6 + j] = clampr(u[6 + j], -m->vlim, m->vlim);
  real w2 = u[0] * u[0] + u[1] * u[1] + u[2] * u[2];
  if (w2 > m->wmax * m->wmax) {
    real sc = m->wmax / sqrtr(w2);
    u[0] *= sc; u[1] *= sc; u[2] *= sc;
  }
}

/* the pose integration of a substep over time T with the pose velocity ua (root twist at P) and
 * wv = omega x v_P at the substep start: root origin += T (v + T wv), root orientation by the exact
 * exponential map, joints += T qdot wrapped as PhysX reports them */
static void advance_pose(phys_t* s, const real ua[NV], const real wv[3], real T) {
  for (int a = 0; a < 3; ++a) s->root_pos[a] += T * (ua[3 + a] + T * wv[a]);
  {
    const real* om = ua;
    real th = sqrtr(om[0] * om[0] + om[1] * om[1] + om[2] * om[2]) * T;
    real dq[4];
    if (th > (real)1e-12) {
      real sc = (real)sin((double)(0.5 * th)) / th * T;
      dq[0] = (real)cos((double)(0.5 * th));
      dq[1] = om[0] * sc; dq[2] = om[1] * sc; dq[3] = om[2] * sc;
    } else {
      dq[0] = 1; dq[1] = (real)0.5 * T * om[0]; dq[2] = (real)0.5 * T * om[1]; dq[3] = (real)0.5 * T * om[2];
    }
    real qn[4];
    q_mul(dq, s->root_quat, qn);
    q_normalize(qn);
    for (int a = 0; a < 4; ++a) s->root_quat[a] = qn[a];
  }
  for (int j = 0; j < ND; ++j) {
    real q = s->jq[j] + T * ua[6 + j];
    /* PhysX reports unlimited revolute joints wrapped to [-2pi, 2pi] (test_articulation.py:19-20) */
    if (q > (real)TWO_PI) q -= (real)(2 * TWO_PI);
    else if (q < -(real)TWO_PI) q += (real)(2 * TWO_PI);
    s->jq[j] = q;
  }
}

/* mu_link / mu_link_d: per-link static / dynamic friction (standup / manager DR; contact
 * coefficient = product, the ground's being cfg->friction / cfg->friction_dynamic), or NULL for
 * the cfg coefficients on every contact */
static void substep(const mdl_t* m, const zb_task_cfg* cfg, phys_t* s, const real target[ND],
                    const real* mu_link, const real* mu_link_d, clist_t* warm, substep_out_t* out) {
  const real dt = cfg->sim_dt;
  kin_t k;
  fk(m, s, &k);

  /* Isaac Lab's reported applied torque: clip(kp (q* - q) - kd qdot, +-effort) */
  for (int j = 0; j < ND; ++j)
    out->applied_torque[j] = clampr(m->kp * (target[j] - s->jq[j]) - m->kd * s->jqd[j], -m->effort, m->effort);

  sinertia I[NB], Ic[NB];
  for (int b = 0; b < NB; ++b) body_sinertia(m, &k, b, &I[b]);
  Ic[NB - 1] = I[NB - 1];
  for (int b = NB - 2; b >= 0; --b) { Ic[b] = I[b]; si_add(&Ic[b], &Ic[b + 1]); }

  real S[ND][6];
  for (int j = 0; j < ND; ++j) {
    real oxa[3];
    v3_cross(k.org[j], k.axis[j], oxa);
    for (int a = 0; a < 3; ++a) { S[j][a] = k.axis[j][a]; S[j][3 + a] = oxa[a]; }
  }

  /* RNEA bias forces (qddot = 0, gravity as base acceleration) */
  real V[NB][6], A[NB][6], f[NB][6];
  body_vel(&k, s, V);
  for (int a = 0; a < 6; ++a) A[0][a] = 0;
  A[0][5] = cfg->gravity;
  for (int j = 0; j < ND; ++j) {
    real cm[6];
    crossm(V[j + 1], S[j], cm);
    for (int a = 0; a < 6; ++a) A[j + 1][a] = A[j][a] + cm[a] * s->jqd[j];
  }
  for (int b = 0; b < NB; ++b) {
    real IA[6], IV[6], cf[6];
    si_mul(&I[b], A[b], IA);
    si_mul(&I[b], V[b], IV);
    crossf(V[b], IV, cf);
    for (int a = 0; a < 6; ++a) f[b][a] = IA[a] + cf[a];
  }
  for (int b = NB - 2; b >= 0; --b)
    for (int a = 0; a < 6; ++a) f[b][a] += f[b + 1][a];
  real Cb[NV];
  for (int a = 0; a < 6; ++a) Cb[a] = f[0][a];
  for (int j = 0; j < ND; ++j) {
    real t = 0;
    for (int a = 0; a < 6; ++a) t += S[j][a] * f[j + 1][a];
    Cb[6 + j] = t;
  }

  /* CRBA */
  real M[NV][NV];
  memset(M, 0, sizeof(M));
  {
    const sinertia* T = &Ic[0];
    M[0][0] = T->I[0]; M[1][1] = T->I[1]; M[2][2] = T->I[2];
    M[1][0] = M[0][1] = T->I[3]; M[2][0] = M[0][2] = T->I[4]; M[2][1] = M[1][2] = T->I[5];
    /* top-right [h]x, bottom-left its transpose */
    real hx = T->h[0], hy = T->h[1], hz = T->h[2];
    real H[3][3] = {{0, -hz, hy}, {hz, 0, -hx}, {-hy, hx, 0}};
    for (int i = 0; i < 3; ++i)
      for (int j = 0; j < 3; ++j) { M[i][3 + j] = H[i][j]; M[3 + j][i] = H[i][j]; }
    M[3][3] = M[4][4] = M[5][5] = T->m;
  }
  for (int kk = 0; kk < ND; ++kk) {
    real F[6];
    si_mul(&Ic[kk + 1], S[kk], F);
    for (int a = 0; a < 6; ++a) { M[a][6 + kk] = F[a]; M[6 + kk][a] = F[a]; }
    for (int jj = 0; jj <= kk; ++jj) {
      real t = 0;
      for (int a = 0; a < 6; ++a) t += S[jj][a] * F[a];
      M[6 + jj][6 + kk] = t;
      M[6 + kk][6 + jj] = t;
    }
  }

  /* implicit PD drive, pass 1 (all implicit) / pass 2 (saturated joints explicit) */
  const real arm = dt * (m->kd + dt * m->kp);
  real u[NV];
  for (int a = 0; a < 3; ++a) { u[a] = s->root_angvel[a]; u[3 + a] = s->root_linvel[a]; }
  for (int j = 0; j < ND; ++j) u[6 + j] = s->jqd[j];
  real rhs_impl[ND];
  for (int j = 0; j < ND; ++j)
    rhs_impl[j] = m->kp * (target[j] - s->jq[j]) - (m->kd + dt * m->kp) * s->jqd[j];

  real L[NV][NV], w[NV], Mw[NV][NV];
  int sat[ND] = {0, 0, 0, 0, 0, 0};
  real sat_tau[ND] = {0, 0, 0, 0, 0, 0};
  for (int pass = 0; pass < 2; ++pass) {
    memcpy(Mw, M, sizeof(M));
    real b[NV];
    for (int a = 0; a < 6; ++a) b[a] = -dt * Cb[a];
    for (int j = 0; j < ND; ++j) {
      if (sat[j]) {
        b[6 + j] = dt * (sat_tau[j] - Cb[6 + j]);
      } else {
        Mw[6 + j][6 + j] += arm;
        b[6 + j] = dt * (rhs_impl[j] - Cb[6 + j]);
      }
    }
    cholesky(Mw, L);
    real z[NV];
    lt_mul(L, u, w);
    fwd_sub(L, b, z);
    for (int a = 0; a < NV; ++a) w[a] += z[a];
    if (pass == 1) break;
    real uf[NV];
    bwd_sub(L, w, uf);
    int any = 0;
    for (int j = 0; j < ND; ++j) {
      real tau = rhs_impl[j] - (arm / dt) * (uf[6 + j] - s->jqd[j]);
      if (tau > m->effort || tau < -m->effort) { sat[j] = 1; sat_tau[j] = tau > 0 ? m->effort : -m->effort; any = 1; }
    }
    if (!any) break;
  }

  /* contacts */
  clist_t CL;
  detect(m, cfg, &k, s->root_pos[2], warm, &CL);
  int nc = CL.n;
  if (warm) *warm = CL; /* the next substep of this step warm-starts GJK from these normals */
  real Y[NC_MAX][3][NV];
  real invm[NC_MAX][3], vmin[NC_MAX], lam[NC_MAX][3], c01[NC_MAX], c02[NC_MAX], muc[NC_MAX], mud[NC_MAX];
  /* TGS-style solve (cfg->solver_mode 1): solver_iterations sub-iterations of h = dt / iterations;
   * sepc = each contact's separation advanced by h times its normal velocity after every
   * sub-iteration (the bias re-linearised), wsum = the sum of the sub-iterations' w.
   * solver_mode 2 adds the per-position-iteration refresh of the ground contacts (PhysX TGS,
   * zbot_cfg.py:637-638): before sub-iteration it > 0 the pose is advanced by it * h with the mean
   * velocity of the sub-iterations so far (the same integration as the substep's end), and every
   * ground contact's point (its rim candidate re-supported at that pose), separation and Jacobian
   * rows are re-evaluated there; the mass matrix and its factor stay the substep's, the rows
   * keep mapping the root twist at the substep's P. Self contacts keep mode 1's linear advance;
   * solver_mode 3 refreshes them too: each self contact's two body-fixed anchors (placed so that
   * n.(pa - pb) is the detected separation) are carried to the advanced pose, the separation is
   * n.(pa' - pb') along the substep's normal and the rows are re-evaluated at their midpoint. */
  const int tgs = cfg->solver_mode >= 1, refresh = cfg->solver_mode >= 2, refresh_self = cfg->solver_mode == 3;
  real wv[3]; /* omega x v_P at the substep start (the classical correction of the root origin) */
  v3_cross(s->root_angvel, s->root_linvel, wv);
  const real h = dt / (real)cfg->solver_iterations;
  real sepc[NC_MAX], wsum[NV];
  for (int a = 0; a < NV; ++a) wsum[a] = 0;
  int broken[NC_MAX];
  real dirs[NC_MAX][3][3];
  real anc[NC_MAX][2][3]; /* solver_mode 3: self contacts' anchors in their bodies' frames */
  int planted = 0;
  for (int c = 0; c < nc; ++c) {
    contact_t* ct = &CL.c[c];
    if (g_plant == 2 && !planted && ct->lb >= 0) {
      for (int a = 0; a < 3; ++a) ct->n[a] = -ct->n[a];
      planted = 1;
    }
    for (int a = 0; a < 3; ++a) dirs[c][0][a] = ct->n[a];
    tangents(ct->n, dirs[c][1], dirs[c][2]);
    /* friction combine mode "multiply" (link x ground, link x link) */
    mud[c] = mu_link_d ? mu_link_d[ct->la] * (ct->lb >= 0 ? mu_link_d[ct->lb] : (real)cfg->friction_dynamic)
                       : (real)cfg->friction_dynamic;
    muc[c] = mu_link ? mu_link[ct->la] * (ct->lb >= 0 ? mu_link[ct->lb] : (real)cfg->friction) : (real)cfg->friction;
    if (muc[c] < mud[c]) muc[c] = mud[c]; /* static raised to dynamic (PhysX material combine) */
    if (g_plant == 1 && !planted && ct->lb < 0) { muc[c] *= (real)1.1; mud[c] *= (real)1.1; planted = 1; }
    for (int r = 0; r < 3; ++r) {
      real J[NV], Jb[NV];
      jac_row(&k, m->link_body[ct->la], ct->x, dirs[c][r], J);
      if (ct->lb >= 0) {
        jac_row(&k, m->link_body[ct->lb], ct->x, dirs[c][r], Jb);
        for (int a = 0; a < NV; ++a) J[a] -= Jb[a];
      }
      fwd_sub(L, J, Y[c][r]);
      real yy = 0;
      for (int a = 0; a < NV; ++a) yy += Y[c][r][a] * Y[c][r][a];
      invm[c][r] = (real)1 / (yy + (real)1e-9);
      lam[c][r] = 0;
    }
    c01[c] = 0; c02[c] = 0;
    broken[c] = 0;
    for (int a = 0; a < NV; ++a) { c01[c] += Y[c][1][a] * Y[c][0][a]; c02[c] += Y[c][2][a] * Y[c][0][a]; }
    sepc[c] = ct->sep;
    vmin[c] = contact_bias(cfg, m, sepc[c], tgs ? h : dt, dt);
    if (refresh_self && ct->lb >= 0) {
      /* self contact: body-fixed anchors pa = x + n sep / 2 on A, pb = x - n sep / 2 on B (so
       * n.(pa - pb) = sep at this pose), kept in the bodies' frames for the refresh */
      const int bs[2] = {m->link_body[ct->la], m->link_body[ct->lb]};
      for (int e = 0; e < 2; ++e) {
        const real* R = k.R[bs[e]];
        real d[3];
        for (int a = 0; a < 3; ++a) d[a] = ct->x[a] + (e ? -(real)0.5 : (real)0.5) * ct->sep * ct->n[a] - k.p[bs[e]][a];
        for (int a = 0; a < 3; ++a) anc[c][e][a] = R[a] * d[0] + R[3 + a] * d[1] + R[6 + a] * d[2];
      }
    }
  }
  /* Gauss-Seidel over contacts; the three row dots of a contact use the same w, the normal
   * update enters the tangent velocities through the cross terms c01 = Y1.Y0, c02 = Y2.Y0
   * (algebraically the sequential normal-then-friction update). */
  for (int it = 0; it < cfg->solver_iterations; ++it) {
    if (tgs && it > 0)
      for (int c = 0; c < nc; ++c) {
        real vn = 0;
        for (int a = 0; a < NV; ++a) vn += Y[c][0][a] * w[a];
        sepc[c] += h * vn;
        vmin[c] = contact_bias(cfg, m, sepc[c], h, dt);
      }
    if (refresh && it > 0) {
      real wm[NV], um[NV];
      for (int a = 0; a < NV; ++a) wm[a] = wsum[a] / (real)it;
      bwd_sub(L, wm, um);
      clamp_speeds(m, um);
      phys_t s2 = *s;
      advance_pose(&s2, um, wv, (real)it * h);
      kin_t k2;
      fk(m, &s2, &k2);
      real dP[3]; /* k2 relative to the substep's P: the rows keep the substep's root reference */
      for (int a = 0; a < 3; ++a) dP[a] = s2.root_pos[a] - s->root_pos[a];
      for (int b = 0; b < NB; ++b)
        for (int a = 0; a < 3; ++a) k2.p[b][a] += dP[a];
      for (int j = 0; j < ND; ++j)
        for (int a = 0; a < 3; ++a) k2.org[j][a] += dP[a];
      for (int c = 0; c < nc; ++c) {
        const contact_t* ct = &CL.c[c];
        if (ct->lb >= 0 && !refresh_self) continue;
        real x[3];
        if (ct->lb < 0) {
          ground_rim_point(m, &k2, ct->la, ct->rim >> 2, ct->rim & 3, x);
          sepc[c] = s->root_pos[2] + x[2];
        } else {
          /* the anchors at the advanced pose: separation n.(pa' - pb') along the substep's normal,
           * the rows at their midpoint */
          real pe[2][3];
          const int bs[2] = {m->link_body[ct->la], m->link_body[ct->lb]};
          for (int e = 0; e < 2; ++e) {
            m3_v(k2.R[bs[e]], anc[c][e], pe[e]);
            for (int a = 0; a < 3; ++a) pe[e][a] += k2.p[bs[e]][a];
          }
          sepc[c] = 0;
          for (int a = 0; a < 3; ++a) {
            sepc[c] += ct->n[a] * (pe[0][a] - pe[1][a]);
            x[a] = (real)0.5 * (pe[0][a] + pe[1][a]);
          }
        }
        for (int r = 0; r < 3; ++r) {
          real J[NV];
          jac_row(&k2, m->link_body[ct->la], x, dirs[c][r], J);
          if (ct->lb >= 0) {
            real Jb[NV];
            jac_row(&k2, m->link_body[ct->lb], x, dirs[c][r], Jb);
            for (int a = 0; a < NV; ++a) J[a] -= Jb[a];
          }
          fwd_sub(L, J, Y[c][r]);
          real yy = 0;
          for (int a = 0; a < NV; ++a) yy += Y[c][r][a] * Y[c][r][a];
          invm[c][r] = (real)1 / (yy + (real)1e-9);
        }
        c01[c] = 0; c02[c] = 0;
        for (int a = 0; a < NV; ++a) { c01[c] += Y[c][1][a] * Y[c][0][a]; c02[c] += Y[c][2][a] * Y[c][0][a]; }
        vmin[c] = contact_bias(cfg, m, sepc[c], h, dt);
      }
    }
    for (int c = 0; c < nc; ++c) {
      const real mu = muc[c];
      real vn = 0, v1 = 0, v2 = 0;
      for (int a = 0; a < NV; ++a) { vn += Y[c][0][a] * w[a]; v1 += Y[c][1][a] * w[a]; v2 += Y[c][2][a] * w[a]; }
      real ln = lam[c][0] + (vmin[c] - vn) * invm[c][0];
      if (ln < 0) ln = 0;
      real dl = ln - lam[c][0];
      real vt1 = v1 + c01[c] * dl, vt2 = v2 + c02[c] * dl;
      real l1 = lam[c][1] - vt1 * invm[c][1];
      real l2 = lam[c][2] - vt2 * invm[c][2];
      /* static / dynamic Coulomb disk (PhysX patch friction): sticks while |l| <= mu_s ln; once a
       * loaded contact (ln > 0) exceeds the static cone it is broken for the rest of this
       * substep's sweeps and slides with |l| = mu_d ln (mu_d = mu_s: the plain disk projection);
       * an unloaded contact's friction is projected to 0 without breaking it */
      real mag2 = l1 * l1 + l2 * l2;
      const int over = mag2 > (mu * ln) * (mu * ln);
      if (!broken[c] && over && ln > 0) broken[c] = 1;
      if (broken[c] || over) {
        real lim = (broken[c] ? mud[c] : mu) * ln;
        if (mag2 > lim * lim) {
          real sc = lim / sqrtr(mag2);
          l1 *= sc; l2 *= sc;
        }
      }
      real d1 = l1 - lam[c][1], d2 = l2 - lam[c][2];
      lam[c][0] = ln; lam[c][1] = l1; lam[c][2] = l2;
      for (int a = 0; a < NV; ++a) w[a] += Y[c][0][a] * dl + Y[c][1][a] * d1 + Y[c][2][a] * d2;
    }
    for (int a = 0; a < NV; ++a) wsum[a] += w[a];
  }
  if (t_act)
    for (int c = 0; c < nc; ++c)
      if (lam[c][0] > 0) ++t_act[CL.c[c].lb >= 0];
  real un[NV], ua[NV]; /* the new velocity; the pose integrates ua (TGS: the sub-iterations' mean) */
  bwd_sub(L, w, un);
  if (tgs) {
    for (int a = 0; a < NV; ++a) wsum[a] /= (real)cfg->solver_iterations;
    bwd_sub(L, wsum, ua);
  }

  /* net contact force per link */
  for (int l = 0; l < NL; ++l) out->net_force[l][0] = out->net_force[l][1] = out->net_force[l][2] = 0;
  for (int c = 0; c < nc; ++c) {
    const contact_t* ct = &CL.c[c];
    for (int a = 0; a < 3; ++a) {
      real F = (lam[c][0] * dirs[c][0][a] + lam[c][1] * dirs[c][1][a] + lam[c][2] * dirs[c][2][a]) / dt;
      F *= (real)g_sensor_force_scale;
      out->net_force[ct->la][a] += F;
      if (ct->lb >= 0) out->net_force[ct->lb][a] -= F;
    }
  }

  /* joint speed limit (PhysX max joint velocity = actuator velocity_limit) and root link angular
   * speed limit (RigidBodyPropertiesCfg.max_angular_velocity, zbot_cfg.py:632), on both */
  clamp_speeds(m, un);
  if (tgs) clamp_speeds(m, ua);
  else memcpy(ua, un, sizeof(un));

  /* semi-implicit Euler. u holds the root twist at the fixed point P; the root origin's
   * classical acceleration adds omega x v_P (spatial -> classical). */
  advance_pose(s, ua, wv, dt);
  for (int a = 0; a < 3; ++a) {
    s->root_angvel[a] = un[a];
    s->root_linvel[a] = un[3 + a] + dt * wv[a];
  }
  for (int j = 0; j < ND; ++j) s->jqd[j] = un[6 + j];
}

/* ------------------------------------------------------------------------- MDP pieces */
/* cached kinematics of v2 _get_observations (v2.py:315-345), from a physics state */
typedef struct {
  real base_pos[3], base_quat[4], fwd[3], heading_err, vfwd;
  real feet_pos[2][3], feet_z[2][3], feet_x[2][3];
} obs_cache_t;

static void quat_apply(const real q[4], const real v[3], real o[3]) {
  real R[9];
  q_to_mat(q, R);
  m3_v(R, v, o);
}

/* fills the cache from base/feet link poses and the base COM velocity (all world) */
static void make_cache(const real base_pos[3], const real base_quat[4], const real feet_pos[2][3],
                       const real feet_quat[2][4], const real base_com_vel[3], obs_cache_t* o) {
  static const real zax[3] = {0, 0, 1}, xax[3] = {1, 0, 0}, mzax[3] = {0, 0, -1};
  static const real g[3] = {0, 0, -1}; /* GRAVITY_VEC_W: normalised gravity direction */
  real sh[3];
  for (int a = 0; a < 3; ++a) o->base_pos[a] = base_pos[a];
  for (int a = 0; a < 4; ++a) o->base_quat[a] = base_quat[a];
  quat_apply(base_quat, zax, sh);            /* v2.py:322 */
  v3_cross(g, sh, o->fwd);                   /* v2.py:323 */
  o->heading_err = -o->fwd[1];               /* v2.py:324 */
  o->vfwd = v3_dot(base_com_vel, o->fwd);    /* v2.py:326-327 */
  for (int f = 0; f < 2; ++f) {
    for (int a = 0; a < 3; ++a) o->feet_pos[f][a] = feet_pos[f][a];
    quat_apply(feet_quat[f], f == 0 ? zax : mzax, o->feet_z[f]); /* v2.py:341-344 */
    quat_apply(feet_quat[f], xax, o->feet_x[f]);                 /* v2.py:338-345 */
  }
}

static void cache_from_phys(const mdl_t* m, const phys_t* s, obs_cache_t* o) {
  kin_t k;
  fk(m, s, &k);
  real V[NB][6];
  body_vel(&k, s, V);
  real bp[3], bq[4], fp[2][3], fq[2][4], bv[3], c[3];
  link_pose(m, &k, m->base_link, bp, bq);
  for (int f = 0; f < 2; ++f) link_pose(m, &k, m->foot_links[f], fp[f], fq[f]);
  int bb = m->link_body[m->base_link];
  m3_v(k.R[bb], m->link_com[m->base_link], c);
  for (int a = 0; a < 3; ++a) c[a] += k.p[bb][a];
  point_vel(V[bb], c, bv);
  for (int a = 0; a < 3; ++a) {
    bp[a] += s->root_pos[a];
    fp[0][a] += s->root_pos[a];
    fp[1][a] += s->root_pos[a];
  }
  make_cache(bp, bq, fp, fq, bv, o);
}

/* post-step quantities the reward/done terms read directly from the sim (no lag) */
typedef struct {
  real jq[ND], jqd[ND], applied_torque[ND];
  real feet_vel[2][3];              /* body_com_lin_vel_w of the feet */
  real feet_fz_hist[ZB_HIST][2];    /* sensor history, slot 0 newest */
  real undes_fmax_hist[ZB_HIST];
  real feet_air_last[2];
  int32_t ep_len;                   /* after the += 1 */
  real origin_y;
} post_t;

/* _get_dones (v2.py:384-411) + _get_rewards (v2.py:371-382, terms 461-561). Updates the MDP
 * integrators in `md`; returns reward; terms[] receives the scaled per-term rewards. */
static real mdp_eval(const zb_task_cfg* cfg, const real jq0[ND], const obs_cache_t* pre,
                     const post_t* ps, mdp_t* md, const real act[ND], const real prev_act[ND],
                     real terms[ZB_NUM_REWARD_TERMS], int* died_out, int* timeout_out) {
  /* ---- dones */
  int time_out = ps->ep_len >= cfg->max_episode_length - 1;
  real feetF[2];
  for (int f = 0; f < 2; ++f) {
    real s = 0;
    for (int h = 0; h < ZB_HIST; ++h) s += ps->feet_fz_hist[h][f];
    feetF[f] = s / (real)ZB_HIST;                          /* v2.py:387-390 */
  }
  int died = 0;
  for (int h = 0; h < ZB_HIST; ++h) died |= ps->undes_fmax_hist[h] > (real)1.0; /* v2.py:396-402 */
  died |= pre->base_pos[2] < cfg->termination_height;      /* v2.py:405 */
  real base_y_err = pre->base_pos[1] - ps->origin_y;       /* v2.py:406 */
  died |= fabs((double)base_y_err) > 0.5;                  /* v2.py:407 */

  /* ---- rewards in dict order */
  const float* sc = cfg->reward_scales;
  real r[ZB_NUM_REWARD_TERMS];
  r[ZB_R_BASE_VEL_FORWARD] = (real)tanh((double)(10 * pre->vfwd / cfg->joint_speed_limit));
  {
    real s = 0;
    for (int f = 0; f < 2; ++f) {
      real d[3] = {pre->feet_z[f][0], pre->feet_z[f][1], pre->feet_z[f][2] - 1};
      s += sqrtr(v3_dot(d, d));
    }
    r[ZB_R_FEET_DOWNWARD] = s;
  }
  {
    real s = 0;
    for (int f = 0; f < 2; ++f) {
      real d[3] = {pre->feet_x[f][0] - pre->fwd[0], pre->feet_x[f][1] - pre->fwd[1], pre->feet_x[f][2] - pre->fwd[2]};
      s += sqrtr(v3_dot(d, d));
    }
    r[ZB_R_FEET_FORWARD] = s;
  }
  r[ZB_R_BASE_HEADING_X] = (real)fabs((double)pre->heading_err);
  /* a stateful term's buffers advance only while it is in the active reward_cfg: the reference
   * updates them inside _reward_<name>, which exists only for the cfg's keys (v2.py:249-252) */
  const uint32_t on = cfg->reward_active;
  if ((on >> ZB_R_BASE_HEADING_X_SUM) & 1u)
    md->heading_sum = clampr(md->heading_sum + (real)0.01 * pre->heading_err, -1, 1);
  r[ZB_R_BASE_HEADING_X_SUM] = (real)fabs((double)md->heading_sum);
  {
    /* step_length v2.py:509-533 */
    const int step_on = (on >> ZB_R_STEP_LENGTH) & 1u;
    real minlen = 0;
    for (int f = 0; f < 2; ++f) {
      int down = step_on && feetF[f] > (real)10.0 && md->feet_f_last[f] < (real)10.0;
      if (down) {
        real d[3] = {pre->feet_pos[f][0] - md->feet_down_pos[f][0], pre->feet_pos[f][1] - md->feet_down_pos[f][1],
                     pre->feet_pos[f][2] - md->feet_down_pos[f][2]};
        md->feet_step_len[f] = v3_dot(d, pre->fwd);
        for (int a = 0; a < 3; ++a) md->feet_down_pos[f][a] = pre->feet_pos[f][a];
      }
    }
    minlen = md->feet_step_len[0] < md->feet_step_len[1] ? md->feet_step_len[0] : md->feet_step_len[1];
    if (step_on) {  /* v2.py:532 */
      md->feet_f_last[0] = feetF[0];
      md->feet_f_last[1] = feetF[1];
    }
    r[ZB_R_STEP_LENGTH] = (real)tanh((double)(15 * minlen));
  }
  r[ZB_R_AIRTIME_BALANCE] = (real)fabs((double)(ps->feet_air_last[0] - ps->feet_air_last[1]));
  {
    real s = 0;
    for (int j = 0; j < ND; ++j) { real d = act[j] - prev_act[j]; s += d * d; }
    r[ZB_R_ACTION_RATE] = s;
  }
  {
    real s = 0;
    for (int j = 0; j < ND; ++j) s += ps->applied_torque[j] * ps->applied_torque[j];
    r[ZB_R_TORQUES] = s;
  }
  {
    real s = 0;
    for (int f = 0; f < 2; ++f) {
      real v = sqrtr(ps->feet_vel[f][0] * ps->feet_vel[f][0] + ps->feet_vel[f][1] * ps->feet_vel[f][1]);
      s += v * (feetF[f] > (real)1.0 ? (real)1 : (real)0);
    }
    r[ZB_R_FEET_SLIDE] = s;
  }
  r[ZB_R_BASE_POS_Y_ERR] = (real)fabs((double)(pre->feet_pos[0][1] + pre->feet_pos[1][1] - 2 * ps->origin_y)) +
                           (real)fabs((double)(pre->base_pos[1] - ps->origin_y));
  if ((on >> ZB_R_BASE_POS_Y_ERR_SUM) & 1u) md->yerr_sum = clampr(md->yerr_sum + (real)0.01 * base_y_err, -1, 1);
  r[ZB_R_BASE_POS_Y_ERR_SUM] = (real)fabs((double)md->yerr_sum);
  r[ZB_R_AIRTIME_SUM] = (real)tanh((double)(ps->feet_air_last[0] + ps->feet_air_last[1]));
  /* step0 (v2.py:563-571, dict order diff before sum): the difference is signed by the integrator
   * before this step's update; torch.sign(0) = 0 */
  r[ZB_R_FEET_FORCE_DIFF] = (feetF[1] - feetF[0]) *
                            (md->force_sum > 0 ? (real)1 : (md->force_sum < 0 ? (real)-1 : (real)0));
  if ((on >> ZB_R_FEET_FORCE_SUM) & 1u) md->force_sum = md->force_sum + (real)0.001 * (feetF[0] - feetF[1]);
  r[ZB_R_FEET_FORCE_SUM] = (real)fabs((double)md->force_sum);

  real rew = 0;
  for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) {
    real v = r[t] * sc[t];
    terms[t] = v;
    rew += v;
    md->ep_sums[t] += v;
  }
  if (died) rew -= cfg->terminal_penalty;  /* v2.py:379-380 */
  (void)jq0;
  *died_out = died;
  *timeout_out = time_out;
  return rew;
}

/* ContactSensor.update after every physics step (history_length > 0 makes Isaac Lab's
 * SensorBase.update refresh the buffers each scene.update(physics_dt)): history roll, air/contact
 * timers with elapsed = sim_dt, is_contact = |F| > threshold. */
static void sensor_update(const mdl_t* m, const zb_task_cfg* cfg, mdp_t* md, const real F[NL][3]) {
  for (int h = ZB_HIST - 1; h > 0; --h) {
    md->feet_fz_hist[h][0] = md->feet_fz_hist[h - 1][0];
    md->feet_fz_hist[h][1] = md->feet_fz_hist[h - 1][1];
    md->undes_fmax_hist[h] = md->undes_fmax_hist[h - 1];
  }
  real fmax = 0;
  for (int k = 0; k < 10; ++k) {
    const real* f = F[m->undesired[k]];
    real nrm = sqrtr(v3_dot(f, f));
    if (nrm > fmax) fmax = nrm;
  }
  md->undes_fmax_hist[0] = fmax;
  const real el = cfg->sim_dt;
  for (int f = 0; f < 2; ++f) {
    const real* Ff = F[m->foot_links[f]];
    md->feet_fz_hist[0][f] = Ff[2];
    int contact = sqrtr(v3_dot(Ff, Ff)) > cfg->contact_force_threshold;
    int first_contact = md->feet_air_cur[f] > 0 && contact;
    if (first_contact) md->feet_air_last[f] = md->feet_air_cur[f] + el;
    md->feet_air_cur[f] = contact ? 0 : md->feet_air_cur[f] + el;
    md->feet_contact_cur[f] = contact ? md->feet_contact_cur[f] + el : 0;
  }
}

/* default physical state (reset pose) */
static void phys_default(const mdl_t* m, phys_t* s) {
  for (int a = 0; a < 3; ++a) { s->root_pos[a] = m->root_pos0[a]; s->root_linvel[a] = 0; s->root_angvel[a] = 0; }
  for (int a = 0; a < 4; ++a) s->root_quat[a] = m->root_quat0[a];
  for (int j = 0; j < ND; ++j) { s->jq[j] = m->jq0[j]; s->jqd[j] = 0; }
}

/* feet link origins (world = env-local) of a physical state */
static void feet_world(const mdl_t* m, const phys_t* ph, real out[2][3]) {
  kin_t k;
  fk(m, ph, &k);
  for (int f = 0; f < 2; ++f) {
    real p[3], q[4];
    link_pose(m, &k, m->foot_links[f], p, q);
    for (int a = 0; a < 3; ++a) out[f][a] = p[a] + ph->root_pos[a];
  }
}

/* feet_down_pos_last on reset (v2.py:436, v4.py:996, mdp/rewards.py:42): the reference reads
 * body_link_pos_w inside _reset_idx, after write_*_to_sim but before DirectRLEnv.step's
 * sim.forward(), so PhysX still reports the pre-reset link transforms: the latch takes the
 * pre-reset (terminal) feet positions `pre`. cfg->reset_feet_refresh = 1 takes the post-reset
 * feet instead (Isaac Lab behaviour, unpinned by any reference artefact). */
static void latch_feet(const mdl_t* m, const zb_task_cfg* cfg, const real pre[2][3], const phys_t* post,
                       real out[2][3]) {
  if (cfg->reset_feet_refresh) {
    feet_world(m, post, out);
  } else {
    for (int f = 0; f < 2; ++f)
      for (int a = 0; a < 3; ++a) out[f][a] = pre[f][a];
  }
}

/* _reset_idx for one env (v2.py:413-459); the episode-log accumulation is done by the caller */
static void reset_env(const mdl_t* m, const zb_task_cfg* cfg, env_t* e) {
  real pre[2][3];
  feet_world(m, &e->ph, pre);
  phys_default(m, &e->ph);
  mdp_t* md = &e->md;
  for (int j = 0; j < ND; ++j) { md->p_delta[j] = 0; md->actions[j] = 0; }
  latch_feet(m, cfg, pre, &e->ph, md->feet_down_pos);
  md->heading_sum = 0;
  md->yerr_sum = 0;
  md->force_sum = 0; /* v2.py:437 */
  /* ContactSensor.reset: history and timers zeroed */
  for (int h = 0; h < ZB_HIST; ++h) { md->feet_fz_hist[h][0] = md->feet_fz_hist[h][1] = 0; md->undes_fmax_hist[h] = 0; }
  for (int f = 0; f < 2; ++f) { md->feet_air_cur[f] = md->feet_air_last[f] = md->feet_contact_cur[f] = 0; }
  md->ep_len = 0;
  for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) md->ep_sums[t] = 0;
  /* NOT reset (reference quirk): feet_step_len, feet_f_last */
  wc_invalidate(e->wc); /* the pose jumped: no warm start */
}

static void write_obs(const mdl_t* m, const env_t* e, float* obs) {
  obs_cache_t oc;
  cache_from_phys(m, &e->ph, &oc);
  for (int a = 0; a < 4; ++a) obs[a] = (float)oc.base_quat[a];
  for (int j = 0; j < ND; ++j) {
    obs[4 + j] = (float)(e->ph.jq[j] - m->jq0[j]);
    obs[10 + j] = (float)e->ph.jqd[j];
    obs[16 + j] = (float)e->md.actions[j];
  }
  obs[22] = 1.0f; /* joint_speed_limit (v2.py:243) */
}


/* ========================================================================= stand-up task
 * zbot-6b-standup-v0: reference source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6_standup_env_v0.py
 * (standup.py). Same physics with per-link friction (startup material randomisation), rewards
 * from post-step link states, died on a 5 cm height drop per 50 steps, in-step resets to a
 * random root pose (reset_root_state_uniform), curriculum on common_step_counter. */

static inline real su_u01(uint64_t h) { return (real)((float)(h >> 40) * (1.0f / 16777216.0f)); }

static void pose_from_samples(const mdl_t* m, const real r[4], int body_frame, phys_t* p);

static inline uint64_t env_hash(uint64_t seed, uint64_t ctr, int i) {
  return zb_hash64(seed ^ zb_hash64(ctr * 0x100000001B3ull + (uint64_t)i));
}
static inline real draw(uint64_t h, int k) { return su_u01(zb_hash64(h + 0x632BE59BD9B4E019ull * (uint64_t)k)); }

/* reset_root_state_uniform (standup.py:33-97, v4.py:59-105) from stream h (draws 1..4, same
 * as the kernel); returns the yaw sample (stored as env.current_yaw) */
static real reset_pose(const mdl_t* m, const zb_task_cfg* cfg, uint64_t h, phys_t* p) {
  real r[4];
  for (int k = 0; k < 4; ++k)
    r[k] = draw(h, k + 1) * ((real)cfg->reset_pose_range[k][1] - (real)cfg->reset_pose_range[k][0]) +
           (real)cfg->reset_pose_range[k][0];
  pose_from_samples(m, r, cfg->reset_pose_body_frame, p);
  return r[3];
}

static void su_reset_pose(const mdl_t* m, const zb_task_cfg* cfg, uint64_t seed, uint64_t ctr, int i, phys_t* p) {
  (void)reset_pose(m, cfg, env_hash(seed, ctr, i), p);
}

/* root pose from the samples (x, y, roll, yaw): quat_from_euler_xyz(roll, 0, yaw) applied in the
 * world frame (delta * default, standup.py:87-88) or the body frame (default * delta, v4.py:88) */
static void pose_from_samples(const mdl_t* m, const real r[4], int body_frame, phys_t* p) {
  /* quat_from_euler_xyz(roll, pitch = 0, yaw) (Isaac Lab math: extrinsic X then Z) */
  const real cr = (real)cos(0.5 * (double)r[2]), sr = (real)sin(0.5 * (double)r[2]);
  const real cy = (real)cos(0.5 * (double)r[3]), sy = (real)sin(0.5 * (double)r[3]);
  const real dq[4] = {cy * cr, cy * sr, sy * sr, sy * cr};
  /* the sampled pose is the Isaac Lab root's: its default pose is chain-root default * T
   * (T = api_root_in_root; identity unless the asset is rooted elsewhere, as v09 at the base) */
  real qa0[4], ta[3], R0[9];
  q_mul(m->root_quat0, m->api_q, qa0);
  q_to_mat(m->root_quat0, R0);
  m3_v(R0, m->api_t, ta);
  real qa[4];
  if (body_frame) q_mul(qa0, dq, qa);
  else q_mul(dq, qa0, qa);
  q_normalize(qa);
  const real pa[3] = {m->root_pos0[0] + ta[0] + r[0], m->root_pos0[1] + ta[1] + r[1], m->root_pos0[2] + ta[2]};
  /* back to the chain root: q = qa * conj(qT), p = pa - R(q) tT */
  const real qTc[4] = {m->api_q[0], -m->api_q[1], -m->api_q[2], -m->api_q[3]};
  real qn[4], Rn[9], tq[3];
  q_mul(qa, qTc, qn);
  q_to_mat(qn, Rn);
  m3_v(Rn, m->api_t, tq);
  for (int a = 0; a < 4; ++a) p->root_quat[a] = qn[a];
  for (int a = 0; a < 3; ++a) p->root_pos[a] = pa[a] - tq[a];
  for (int a = 0; a < 3; ++a) { p->root_linvel[a] = 0; p->root_angvel[a] = 0; }
  for (int j = 0; j < ND; ++j) { p->jq[j] = m->jq0[j]; p->jqd[j] = 0; }
}

/* _reset_idx (standup.py:645-703) minus the log: pose event, joints default, p_delta / actions
 * zero, center_z_last 0.05, ep_len 0, episode sums zero; the friction (startup event) stays */
static void su_reset_env(const mdl_t* m, const zb_task_cfg* cfg, uint64_t seed, uint64_t ctr, int i, env_t* e) {
  wc_invalidate(e->wc); /* the pose jumps: no warm start */
  su_reset_pose(m, cfg, seed, ctr, i, &e->ph);
  mdp_t* md = &e->md;
  for (int j = 0; j < ND; ++j) { md->p_delta[j] = 0; md->actions[j] = 0; }
  md->center_z_last = cfg->center_z_init;
  md->ep_len = 0;
  for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) md->ep_sums[t] = 0;
}

/* the stand-up MDP's reads of body_link_state_w: link z heights (4 = a3, 6 = base, 8 = a5),
 * link-origin z velocities (5 = b3, 6), feet link quaternions, base link quaternion */
typedef struct { real z4, z6, z8, vz5, vz6, feet_quat[2][4], base_quat[4]; } su_links_t;

static void su_links(const mdl_t* m, const phys_t* s, su_links_t* o) {
  kin_t k;
  fk(m, s, &k);
  real V[NB][6], p[3], q[4];
  body_vel(&k, s, V);
  link_pose(m, &k, 4, p, q); o->z4 = p[2] + s->root_pos[2];
  link_pose(m, &k, 8, p, q); o->z8 = p[2] + s->root_pos[2];
  link_pose(m, &k, 6, p, o->base_quat); o->z6 = p[2] + s->root_pos[2];
  link_pose(m, &k, m->foot_links[0], p, o->feet_quat[0]);
  link_pose(m, &k, m->foot_links[1], p, o->feet_quat[1]);
  const int ls[2] = {5, 6};
  real* vz[2] = {&o->vz5, &o->vz6};
  for (int t = 0; t < 2; ++t) {
    const int l = ls[t], b = m->link_body[l];
    real x[3], v[3];
    m3_v(k.R[b], m->link_pos[l], x); /* link frame origin: body_link_lin_vel_w */
    for (int a = 0; a < 3; ++a) x[a] += k.p[b][a];
    point_vel(V[b], x, v);
    *vz[t] = v[2];
  }
}

/* _get_dones (634-643) + _get_rewards (620-632; terms upward_2 843-856, shape_symmetry 782-789,
 * feet_downward 735-745, feet_downward_4 827-840). ep_len is after the += 1. Updates
 * center_z_last and the episode sums; returns the reward. */
static real su_mdp_eval(const zb_task_cfg* cfg, int stage, const su_links_t* L, const real pdel[ND], int32_t ep_len,
                        real* center_z_last, real ep_sums[ZB_SU_NUM_REWARD_TERMS], real terms[ZB_SU_NUM_REWARD_TERMS],
                        int* died_out, int* tout_out) {
  static const real zax[3] = {0, 0, 1}, mzax[3] = {0, 0, -1};
  const int time_out = ep_len >= cfg->max_episode_length - 1;
  const int died = (*center_z_last - L->z6) > (real)cfg->center_z_drop;
  if (ep_len % cfg->center_z_period == cfg->center_z_period - 1) *center_z_last = L->z6;
  real fz[2][3];
  quat_apply(L->feet_quat[0], zax, fz[0]);
  quat_apply(L->feet_quat[1], mzax, fz[1]);
  real r[ZB_SU_NUM_REWARD_TERMS];
  {
    const real rh = L->z6 + (real)0.5 * L->z4 + (real)0.5 * L->z8 - (real)0.1f;
    real up = L->z6 < (real)0.22f ? rh + (real)0.5 * L->vz6 + (real)0.5 * L->vz5 : (real)1.35f;
    if ((fz[0][2] < (real)0.5 || fz[1][2] < (real)0.5) && L->z6 > (real)0.1f) up = (real)-5.0 * up;
    r[ZB_SU_R_UPWARD_2] = up;
  }
  r[ZB_SU_R_SHAPE_SYMMETRY] = (real)(fabs((double)(pdel[0] + pdel[5])) + fabs((double)(pdel[1] + pdel[4])) +
                                     fabs((double)(pdel[2] + pdel[3])));
  {
    real sd = 0;
    for (int f = 0; f < 2; ++f) {
      const real d[3] = {fz[f][0], fz[f][1], fz[f][2] - 1};
      sd += sqrtr(v3_dot(d, d));
    }
    r[ZB_SU_R_FEET_DOWNWARD] = sd;
  }
  r[ZB_SU_R_FEET_DOWNWARD_4] = L->z6 < (real)0.15f ? fz[0][2] + fz[1][2] : (real)1.6f;
  const real step_dt = (real)(cfg->sim_dt * (float)cfg->decimation);
  real rew = 0;
  for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) {
    const real w = (real)cfg->stage_scales[stage][t];
    const real v = (r[t] * w) * step_dt;
    terms[t] = v;
    rew += v;
    ep_sums[t] += v;
  }
  if (died) rew -= cfg->terminal_penalty;
  *died_out = died;
  *tout_out = time_out;
  return rew;
}

static void su_write_obs(const mdl_t* m, const env_t* e, float* obs) {
  su_links_t L;
  su_links(m, &e->ph, &L);
  for (int a = 0; a < 4; ++a) obs[a] = (float)L.base_quat[a];
  for (int j = 0; j < ND; ++j) {
    obs[4 + j] = (float)(e->ph.jq[j] - m->jq0[j]);
    obs[10 + j] = (float)e->ph.jqd[j];
    obs[16 + j] = (float)e->md.actions[j];
  }
}

static real su_step_env(const mdl_t* m, const zb_task_cfg* cfg, int stage, uint64_t seed, uint64_t ctr, int i,
                        env_t* e, const float* action, float* obs, int* died, int* tout,
                        real acc[ZB_MAX_REWARD_TERMS]) {
  mdp_t* md = &e->md;
  real act[ND], target[ND];
  const real step_dt = (real)(cfg->sim_dt * (float)cfg->decimation);
  for (int j = 0; j < ND; ++j) { /* _pre_physics_step mode 1 (standup.py:538-551) */
    act[j] = (real)tanh((double)action[j]);
    real pd = md->p_delta[j] + (real)PI_R * act[j] * cfg->joint_speed_limit * step_dt;
    md->p_delta[j] = clampr(pd, -(real)PI_R, (real)PI_R);
    target[j] = md->p_delta[j] + m->jq0[j];
  }
  substep_out_t so;
  clist_t wl;
  wc_warm_list(e->wc, &wl);
  for (int k = 0; k < cfg->decimation; ++k) substep(m, cfg, &e->ph, target, md->mu, md->mu_d, &wl, &so);
  wc_store(&wl, e->wc);
  md->ep_len += 1;
  for (int j = 0; j < ND; ++j) md->actions[j] = act[j];
  su_links_t L;
  su_links(m, &e->ph, &L);
  real terms[ZB_SU_NUM_REWARD_TERMS];
  real rew = su_mdp_eval(cfg, stage, &L, md->p_delta, md->ep_len, &md->center_z_last, md->ep_sums, terms, died, tout);
  if (*died || *tout) {
    /* Episode_Reward/<term> = mean over reset envs of sum / max(ep_len * step_dt, step_dt) (653-659) */
    real dur = (real)md->ep_len * step_dt;
    if (dur < step_dt) dur = step_dt;
    for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) acc[t] += md->ep_sums[t] / dur;
    su_reset_env(m, cfg, seed, ctr, i, e);
  }
  su_write_obs(m, e, obs);
  return rew;
}

static void su_pack_env(const env_t* e, float* st, int n, int i) {
#define PUT(off, val) st[(size_t)(off) * n + i] = (float)(val)
  for (int a = 0; a < 3; ++a) { PUT(ZB_S_ROOT_POS + a, e->ph.root_pos[a]); PUT(ZB_S_ROOT_LINVEL + a, e->ph.root_linvel[a]); PUT(ZB_S_ROOT_ANGVEL + a, e->ph.root_angvel[a]); }
  for (int a = 0; a < 4; ++a) PUT(ZB_S_ROOT_QUAT + a, e->ph.root_quat[a]);
  for (int j = 0; j < ND; ++j) {
    PUT(ZB_S_JOINT_POS + j, e->ph.jq[j]); PUT(ZB_S_JOINT_VEL + j, e->ph.jqd[j]);
    PUT(ZB_SU_P_DELTA + j, e->md.p_delta[j]); PUT(ZB_SU_ACTIONS + j, e->md.actions[j]);
  }
  PUT(ZB_SU_CENTER_Z_LAST, e->md.center_z_last);
  PUT(ZB_SU_EP_LEN, e->md.ep_len);
  for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) PUT(ZB_SU_EP_SUMS + t, e->md.ep_sums[t]);
  for (int l = 0; l < NL; ++l) { PUT(ZB_SU_LINK_MU + l, e->md.mu[l]); PUT(ZB_SU_LINK_MU_D + l, e->md.mu_d[l]); }
#undef PUT
}
static void su_unpack_env(env_t* e, const float* st, int n, int i) {
#define GET(off) ((real)st[(size_t)(off) * n + i])
  for (int a = 0; a < 3; ++a) { e->ph.root_pos[a] = GET(ZB_S_ROOT_POS + a); e->ph.root_linvel[a] = GET(ZB_S_ROOT_LINVEL + a); e->ph.root_angvel[a] = GET(ZB_S_ROOT_ANGVEL + a); }
  for (int a = 0; a < 4; ++a) e->ph.root_quat[a] = GET(ZB_S_ROOT_QUAT + a);
  for (int j = 0; j < ND; ++j) {
    e->ph.jq[j] = GET(ZB_S_JOINT_POS + j); e->ph.jqd[j] = GET(ZB_S_JOINT_VEL + j);
    e->md.p_delta[j] = GET(ZB_SU_P_DELTA + j); e->md.actions[j] = GET(ZB_SU_ACTIONS + j);
  }
  e->md.center_z_last = GET(ZB_SU_CENTER_Z_LAST);
  e->md.ep_len = (int32_t)lrint((double)st[(size_t)ZB_SU_EP_LEN * n + i]);
  for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) e->md.ep_sums[t] = GET(ZB_SU_EP_SUMS + t);
  for (int l = 0; l < NL; ++l) { e->md.mu[l] = GET(ZB_SU_LINK_MU + l); e->md.mu_d[l] = GET(ZB_SU_LINK_MU_D + l); }
#undef GET
}

/* ========================================================================= walking v4
 * zbot-6b-walking-v4: reference source/zbot/zbot/tasks/zbot6b_direct/zbot_direct_6dof_bipedal_env_v4.py
 * (v4.py). v2's robot and physics; commands (forward velocity, relative yaw) resampled by reset
 * and interval events; a history-3 contact sensor with contact-time tracking; 15 reward terms on
 * the post-step state; my_curriculum (stage weights, command sign probability) and
 * range_curriculum (command ranges). */

static real wrap_to_pi_r(real x) { /* isaaclab.utils.math.wrap_to_pi */
  double a = fmod((double)x, TWO_PI);
  if (a < 0) a += TWO_PI;
  return (real)(a > PI_R ? a - TWO_PI : a);
}

/* resample_commands (v4.py:107-135) on uniform draws (u_sign < prob_pos: Bernoulli sign) */
static void v4_commands(int dual_sign, real prob_pos, const float vr[2], const float yr[2], real offset, real u_sign,
                        real u_vel, real u_yaw, real cur_yaw, real cmd[2], real* target) {
  const real lo = vr[0], hi0 = vr[1];
  if (dual_sign) {
    const real sg = u_sign < prob_pos ? 1 : -1; /* bernoulli(prob_pos) * 2 - 1 */
    const real hi = hi0 + offset * (sg - 1);
    cmd[0] = (u_vel * (hi - lo) + lo) * sg;
  } else {
    cmd[0] = u_vel * (hi0 - lo) + lo;
  }
  cmd[1] = u_yaw * ((real)yr[1] - (real)yr[0]) + (real)yr[0];
  *target = wrap_to_pi_r(cur_yaw + cmd[1]);
}

/* the same with draws k0 .. k0+2 of stream h and the sim's current params */
static void v4_resample(const zbo_sim* s, uint64_t h, int k0, real cur_yaw, real cmd[2], real* target) {
  v4_commands(s->c.cmd_dual_sign, (real)s->prob_pos, s->vel, s->yaw, (real)s->c.cmd_offset, draw(h, k0),
              draw(h, k0 + 1), draw(h, k0 + 2), cur_yaw, cmd, target);
}

/* what the v4 MDP reads after the physics (Isaac Lab data names) */
typedef struct {
  real base_pos[3], base_quat[4], base_lin_vel[3];  /* body_link_*_w[base] */
  real feet_pos[2][3], feet_quat[2][4], feet_com_vel[2][3];
  real jqd[ND], joint_acc[ND], applied_torque[ND];
  real fz_hist[ZB_V4_HIST][2];     /* net_forces_w_history[..., feet, 2], slot 0 newest */
  real undes_fmax_hist[ZB_V4_HIST];/* max over undesired bodies of |net force| per slot */
  real air_cur[2], con_cur[2], air_last[2], con_last[2]; /* sensor timers after the update */
  int32_t ep_len;                  /* after the += 1 */
} v4_post_t;

typedef struct { real cur_yaw, heading_err; } v4_aux_t;

/* _get_dones (896-918) + _get_rewards (883-894; terms 1003-1171 in dict order) with the
 * intermediate values of 809-849. Updates the step-length state and the episode sums. */
static real v4_mdp_eval(const zb_task_cfg* cfg, int stage, const v4_post_t* P, mdp_t* md, const real act[ND],
                        const real prev[ND], real terms[ZB_V4_NUM_REWARD_TERMS], int* died_out, int* tout_out,
                        v4_aux_t* aux) {
  static const real zax[3] = {0, 0, 1}, mzax[3] = {0, 0, -1}, xax[3] = {1, 0, 0};
  const int time_out = P->ep_len >= cfg->max_episode_length - 1;
  real fm = 0;
  for (int h = 0; h < ZB_V4_HIST; ++h) fm = P->undes_fmax_hist[h] > fm ? P->undes_fmax_hist[h] : fm;
  const int died = fm > (real)cfg->undesired_force_threshold || P->base_pos[2] < (real)cfg->termination_height;
  real sh[3], fwd[3];
  quat_apply(P->base_quat, zax, sh);
  fwd[0] = sh[1]; fwd[1] = -sh[0]; fwd[2] = 0; /* GRAVITY_VEC_W (0,0,-1) x shoulder */
  const real cur_yaw = (real)atan2((double)fwd[1], (double)fwd[0]);
  const real d = md->target_yaw - cur_yaw;
  const real he = (real)atan2(sin((double)d), cos((double)d));
  const real vfwd = v3_dot(P->base_lin_vel, fwd);
  real feetF[2];
  for (int f = 0; f < 2; ++f) {
    real a = 0;
    for (int h = 0; h < ZB_V4_HIST; ++h) a += P->fz_hist[h][f];
    feetF[f] = a / (real)ZB_V4_HIST;
  }
  real fz[2][3], fx[2][3];
  for (int f = 0; f < 2; ++f) {
    quat_apply(P->feet_quat[f], f == 0 ? zax : mzax, fz[f]);
    quat_apply(P->feet_quat[f], xax, fx[f]);
  }
  real r[ZB_V4_NUM_REWARD_TERMS];
  {
    const real e = md->commands[0] - vfwd;
    r[ZB_V4_R_TRACK_LIN_VEL_X] = (real)exp(-(double)(e * e) / 0.25);
    r[ZB_V4_R_TRACK_HEADING_YAW] = (real)exp(-(double)(he * he) / 0.25);
    const real vy = v3_dot(P->base_lin_vel, sh);
    r[ZB_V4_R_LIN_VEL_Y] = vy * vy;
    real ar = 0, jv = 0, ja = 0, tq = 0;
    for (int j = 0; j < ND; ++j) {
      ar += (act[j] - prev[j]) * (act[j] - prev[j]);
      jv += P->jqd[j] * P->jqd[j];
      ja += P->joint_acc[j] * P->joint_acc[j];
      tq += P->applied_torque[j] * P->applied_torque[j];
    }
    r[ZB_V4_R_ACTION_RATE] = ar;
    r[ZB_V4_R_TORQUES] = tq;
    r[ZB_V4_R_JOINT_VEL] = jv;
    r[ZB_V4_R_JOINT_ACC] = ja;
    real sd = 0, sf = 0;
    for (int f = 0; f < 2; ++f) {
      const real dz[3] = {fz[f][0], fz[f][1], fz[f][2] - 1};
      sd += sqrtr(v3_dot(dz, dz));
      const real dx[3] = {fx[f][0] - fwd[0], fx[f][1] - fwd[1], fx[f][2] - fwd[2]};
      sf += sqrtr(v3_dot(dx, dx));
    }
    r[ZB_V4_R_FEET_DOWNWARD] = sd;
    r[ZB_V4_R_FEET_FORWARD] = sf;
    /* step_length (1058-1095) */
    const real csg = md->commands[0] > 0 ? 1 : (md->commands[0] < 0 ? -1 : 0);
    for (int f = 0; f < 2; ++f) {
      if (feetF[f] > (real)10.0 && md->feet_f_last[f] < (real)10.0) {
        const real dv[3] = {P->feet_pos[f][0] - md->feet_down_pos[f][0], P->feet_pos[f][1] - md->feet_down_pos[f][1],
                            P->feet_pos[f][2] - md->feet_down_pos[f][2]};
        md->feet_step_len[f] = v3_dot(dv, fwd) * csg;
        for (int a = 0; a < 3; ++a) md->feet_down_pos[f][a] = P->feet_pos[f][a];
      }
    }
    const real mn = md->feet_step_len[0] < md->feet_step_len[1] ? md->feet_step_len[0] : md->feet_step_len[1];
    md->feet_step_len[0] *= (real)0.99f;
    md->feet_step_len[1] *= (real)0.99f;
    md->feet_f_last[0] = feetF[0];
    md->feet_f_last[1] = feetF[1];
    r[ZB_V4_R_STEP_LENGTH] = (real)tanh((double)(15 * mn));
    /* feet_air_time_biped (1129-1143) */
    const int in0 = P->con_cur[0] > 0, in1 = P->con_cur[1] > 0;
    const int single = in0 + in1 == 1;
    real m0 = single ? (in0 ? P->con_cur[0] : P->air_cur[0]) : 0;
    real m1 = single ? (in1 ? P->con_cur[1] : P->air_cur[1]) : 0;
    real bi = m0 < m1 ? m0 : m1;
    r[ZB_V4_R_FEET_AIR_TIME_BIPED] = bi > 2 ? 2 : bi;
    /* airtime_variance (1097-1103): torch.var (unbiased) of two values = (a - b)^2 / 2 */
    const real a0 = P->air_last[0] < (real)0.5 ? P->air_last[0] : (real)0.5;
    const real a1 = P->air_last[1] < (real)0.5 ? P->air_last[1] : (real)0.5;
    const real c0 = P->con_last[0] < (real)0.5 ? P->con_last[0] : (real)0.5;
    const real c1 = P->con_last[1] < (real)0.5 ? P->con_last[1] : (real)0.5;
    r[ZB_V4_R_AIRTIME_VARIANCE] = (real)0.5 * (a0 - a1) * (a0 - a1) + (real)0.5 * (c0 - c1) * (c0 - c1);
    real sl = 0;
    for (int f = 0; f < 2; ++f) {
      const real v = sqrtr(P->feet_com_vel[f][0] * P->feet_com_vel[f][0] + P->feet_com_vel[f][1] * P->feet_com_vel[f][1]);
      sl += v * (feetF[f] > (real)1.0 ? (real)1 : (real)0);
    }
    r[ZB_V4_R_FEET_SLIDE] = sl;
    r[ZB_V4_R_FEET_HARMONY] = (P->air_last[0] + P->air_last[1]) - 3 * (real)fabs((double)(P->air_last[0] - P->air_last[1]));
    const real dx = P->feet_pos[0][0] - P->feet_pos[1][0], dy = P->feet_pos[0][1] - P->feet_pos[1][1];
    const real cl = (real)0.115f - sqrtr(dx * dx + dy * dy);
    r[ZB_V4_R_FEET_CLOSE] = cl > 0 ? cl : 0;
  }
  const real step_dt = (real)(cfg->sim_dt * (float)cfg->decimation);
  real rew = 0;
  for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) {
    const real v = (r[t] * (real)cfg->stage_scales[stage][t]) * step_dt;
    terms[t] = v;
    rew += v;
    md->ep_sums[t] += v;
  }
  if (died) rew -= cfg->terminal_penalty;
  *died_out = died;
  *tout_out = time_out;
  aux->cur_yaw = cur_yaw;
  aux->heading_err = he;
  return rew;
}

/* ContactSensor update (history 3; last_contact_time tracked, v4.py:522-527) */
static void v4_sensor_update(const mdl_t* m, const zb_task_cfg* cfg, mdp_t* md, const real F[NL][3]) {
  for (int h = ZB_V4_HIST - 1; h > 0; --h) {
    md->feet_fz_hist[h][0] = md->feet_fz_hist[h - 1][0];
    md->feet_fz_hist[h][1] = md->feet_fz_hist[h - 1][1];
    md->undes_fmax_hist[h] = md->undes_fmax_hist[h - 1];
  }
  real fmax = 0;
  for (int k = 0; k < 10; ++k) {
    const real* f = F[m->undesired[k]];
    const real nrm = sqrtr(v3_dot(f, f));
    if (nrm > fmax) fmax = nrm;
  }
  md->undes_fmax_hist[0] = fmax;
  const real el = cfg->sim_dt; /* updated every physics step, like sensor_update */
  for (int f = 0; f < 2; ++f) {
    const real* Ff = F[m->foot_links[f]];
    md->feet_fz_hist[0][f] = Ff[2];
    const int c = sqrtr(v3_dot(Ff, Ff)) > cfg->contact_force_threshold;
    if (md->feet_air_cur[f] > 0 && c) md->feet_air_last[f] = md->feet_air_cur[f] + el;
    md->feet_air_cur[f] = c ? 0 : md->feet_air_cur[f] + el;
    if (md->feet_contact_cur[f] > 0 && !c) md->feet_contact_last[f] = md->feet_contact_cur[f] + el;
    md->feet_contact_cur[f] = c ? md->feet_contact_cur[f] + el : 0;
  }
}

/* _reset_idx (920-1001) minus the log: reset events (pose; commands), defaults. init: the
 * construction-time interval timer draw. */
static void v4_reset_env(const zbo_sim* s, uint64_t ctr, int i, env_t* e, int init) {
  wc_invalidate(e->wc); /* the pose jumps: no warm start */
  const mdl_t* m = &s->m;
  const uint64_t h = env_hash(s->seed, ctr, i);
  mdp_t* md = &e->md;
  real pre[2][3];
  feet_world(m, &e->ph, pre);
  md->current_yaw = reset_pose(m, &s->c, h, &e->ph);
  v4_resample(s, h, 5, md->current_yaw, md->commands, &md->target_yaw);
  if (init) md->interval_left = draw(h, 8) * (s->c.cmd_interval_s[1] - s->c.cmd_interval_s[0]) + s->c.cmd_interval_s[0];
  for (int j = 0; j < ND; ++j) { md->p_delta[j] = 0; md->actions[j] = 0; }
  latch_feet(m, &s->c, pre, &e->ph, md->feet_down_pos);
  for (int f = 0; f < 2; ++f) {
    md->feet_f_last[f] = s->c.feet_f_last_init;
    md->feet_step_len[f] = 0;
    md->feet_air_cur[f] = md->feet_air_last[f] = md->feet_contact_cur[f] = md->feet_contact_last[f] = 0;
  }
  for (int h2 = 0; h2 < ZB_HIST; ++h2) { md->feet_fz_hist[h2][0] = md->feet_fz_hist[h2][1] = 0; md->undes_fmax_hist[h2] = 0; }
  md->ep_len = 0;
  for (int t = 0; t < ZB_MAX_REWARD_TERMS; ++t) md->ep_sums[t] = 0;
}

static void v4_write_obs(const mdl_t* m, const env_t* e, float* obs) {
  kin_t k;
  fk(m, &e->ph, &k);
  real p[3], q[4];
  link_pose(m, &k, m->base_link, p, q);
  for (int a = 0; a < 4; ++a) obs[a] = (float)q[a];
  for (int j = 0; j < ND; ++j) {
    obs[4 + j] = (float)(e->ph.jq[j] - m->jq0[j]);
    obs[10 + j] = (float)e->ph.jqd[j];
    obs[16 + j] = (float)e->md.actions[j];
  }
  obs[22] = (float)e->md.commands[0];
  const double d = (double)(e->md.target_yaw - e->md.current_yaw);
  obs[23] = (float)atan2(sin(d), cos(d));
}

static real v4_step_env(const zbo_sim* s, int stage, uint64_t ctr, int i, env_t* e, const float* action, float* obs,
                        int* died, int* tout, real acc[ZB_MAX_REWARD_TERMS]) {
  const mdl_t* m = &s->m;
  const zb_task_cfg* cfg = &s->c;
  mdp_t* md = &e->md;
  real act[ND], prev[ND], target[ND];
  const real step_dt = (real)(cfg->sim_dt * (float)cfg->decimation);
  for (int j = 0; j < ND; ++j) {
    prev[j] = md->actions[j];
    act[j] = (real)tanh((double)action[j]);
    md->p_delta[j] = clampr(md->p_delta[j] + (real)PI_R * act[j] * cfg->joint_speed_limit * step_dt, -(real)PI_R,
                            (real)PI_R);
    target[j] = md->p_delta[j] + m->jq0[j];
  }
  substep_out_t so;
  real jqd_prev[ND];
  clist_t wl;
  wc_warm_list(e->wc, &wl);
  for (int k = 0; k < cfg->decimation; ++k) {
    if (k == cfg->decimation - 1)
      for (int j = 0; j < ND; ++j) jqd_prev[j] = e->ph.jqd[j];
    substep(m, cfg, &e->ph, target, NULL, NULL, &wl, &so);
    v4_sensor_update(m, cfg, md, so.net_force);
  }
  wc_store(&wl, e->wc);
  md->ep_len += 1;
  v4_post_t P;
  {
    kin_t k;
    fk(m, &e->ph, &k);
    real V[NB][6], q[4];
    body_vel(&k, &e->ph, V);
    link_pose(m, &k, m->base_link, P.base_pos, P.base_quat);
    const int bb = m->link_body[m->base_link];
    real x[3];
    m3_v(k.R[bb], m->link_pos[m->base_link], x);
    for (int a = 0; a < 3; ++a) x[a] += k.p[bb][a];
    point_vel(V[bb], x, P.base_lin_vel); /* link-origin velocity */
    for (int a = 0; a < 3; ++a) P.base_pos[a] += e->ph.root_pos[a];
    for (int f = 0; f < 2; ++f) {
      const int l = m->foot_links[f], b = m->link_body[l];
      link_pose(m, &k, l, P.feet_pos[f], P.feet_quat[f]);
      for (int a = 0; a < 3; ++a) P.feet_pos[f][a] += e->ph.root_pos[a];
      real c[3];
      m3_v(k.R[b], m->link_com[l], c);
      for (int a = 0; a < 3; ++a) c[a] += k.p[b][a];
      point_vel(V[b], c, P.feet_com_vel[f]);
    }
    (void)q;
  }
  for (int j = 0; j < ND; ++j) {
    P.jqd[j] = e->ph.jqd[j];
    P.joint_acc[j] = (e->ph.jqd[j] - jqd_prev[j]) / (real)cfg->sim_dt;
    P.applied_torque[j] = so.applied_torque[j];
  }
  for (int h = 0; h < ZB_V4_HIST; ++h) {
    P.fz_hist[h][0] = md->feet_fz_hist[h][0];
    P.fz_hist[h][1] = md->feet_fz_hist[h][1];
    P.undes_fmax_hist[h] = md->undes_fmax_hist[h];
  }
  for (int f = 0; f < 2; ++f) {
    P.air_cur[f] = md->feet_air_cur[f]; P.con_cur[f] = md->feet_contact_cur[f];
    P.air_last[f] = md->feet_air_last[f]; P.con_last[f] = md->feet_contact_last[f];
  }
  P.ep_len = md->ep_len;
  for (int j = 0; j < ND; ++j) md->actions[j] = act[j];
  real terms[ZB_V4_NUM_REWARD_TERMS];
  v4_aux_t aux;
  const real rew = v4_mdp_eval(cfg, stage, &P, md, act, prev, terms, died, tout, &aux);
  md->current_yaw = aux.cur_yaw;
  const uint64_t h = env_hash(s->seed, ctr, i);
  if (*died || *tout) {
    real dur = (real)md->ep_len * step_dt;
    if (dur < step_dt) dur = step_dt;
    for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) acc[t] += md->ep_sums[t] / dur;
    v4_reset_env(s, ctr, i, e, 0);
  }
  /* interval_command_resample (after the resets; v4.py:426-439) */
  md->interval_left -= step_dt;
  if (md->interval_left < (real)1e-6) {
    md->interval_left = draw(h, 8) * (cfg->cmd_interval_s[1] - cfg->cmd_interval_s[0]) + cfg->cmd_interval_s[0];
    v4_resample(s, h, 9, md->current_yaw, md->commands, &md->target_yaw);
  }
  v4_write_obs(m, e, obs);
  return rew;
}

static void v4_pack_env(const env_t* e, float* st, int n, int i) {
#define PUT(off, val) st[(size_t)(off) * n + i] = (float)(val)
  for (int a = 0; a < 3; ++a) { PUT(ZB_S_ROOT_POS + a, e->ph.root_pos[a]); PUT(ZB_S_ROOT_LINVEL + a, e->ph.root_linvel[a]); PUT(ZB_S_ROOT_ANGVEL + a, e->ph.root_angvel[a]); }
  for (int a = 0; a < 4; ++a) PUT(ZB_S_ROOT_QUAT + a, e->ph.root_quat[a]);
  for (int j = 0; j < ND; ++j) {
    PUT(ZB_S_JOINT_POS + j, e->ph.jq[j]); PUT(ZB_S_JOINT_VEL + j, e->ph.jqd[j]);
    PUT(ZB_V4_P_DELTA + j, e->md.p_delta[j]); PUT(ZB_V4_ACTIONS + j, e->md.actions[j]);
  }
  PUT(ZB_V4_COMMANDS, e->md.commands[0]); PUT(ZB_V4_COMMANDS + 1, e->md.commands[1]);
  PUT(ZB_V4_TARGET_YAW, e->md.target_yaw); PUT(ZB_V4_INTERVAL_LEFT, e->md.interval_left);
  PUT(ZB_V4_CURRENT_YAW, e->md.current_yaw);
  for (int f = 0; f < 2; ++f) {
    for (int a = 0; a < 3; ++a) PUT(ZB_V4_FEET_DOWN_POS + 3 * f + a, e->md.feet_down_pos[f][a]);
    PUT(ZB_V4_FEET_STEP_LEN + f, e->md.feet_step_len[f]);
    PUT(ZB_V4_FEET_F_LAST + f, e->md.feet_f_last[f]);
    PUT(ZB_V4_FEET_AIR_CUR + f, e->md.feet_air_cur[f]);
    PUT(ZB_V4_FEET_CONTACT_CUR + f, e->md.feet_contact_cur[f]);
    PUT(ZB_V4_FEET_AIR_LAST + f, e->md.feet_air_last[f]);
    PUT(ZB_V4_FEET_CONTACT_LAST + f, e->md.feet_contact_last[f]);
    for (int h = 0; h < ZB_V4_HIST; ++h) PUT(ZB_V4_FEET_FZ_HIST + 2 * h + f, e->md.feet_fz_hist[h][f]);
  }
  for (int h = 0; h < ZB_V4_HIST; ++h) PUT(ZB_V4_UNDES_FMAX_HIST + h, e->md.undes_fmax_hist[h]);
  PUT(ZB_V4_EP_LEN, e->md.ep_len);
  for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) PUT(ZB_V4_EP_SUMS + t, e->md.ep_sums[t]);
#undef PUT
}
static void v4_unpack_env(env_t* e, const float* st, int n, int i) {
#define GET(off) ((real)st[(size_t)(off) * n + i])
  for (int a = 0; a < 3; ++a) { e->ph.root_pos[a] = GET(ZB_S_ROOT_POS + a); e->ph.root_linvel[a] = GET(ZB_S_ROOT_LINVEL + a); e->ph.root_angvel[a] = GET(ZB_S_ROOT_ANGVEL + a); }
  for (int a = 0; a < 4; ++a) e->ph.root_quat[a] = GET(ZB_S_ROOT_QUAT + a);
  for (int j = 0; j < ND; ++j) {
    e->ph.jq[j] = GET(ZB_S_JOINT_POS + j); e->ph.jqd[j] = GET(ZB_S_JOINT_VEL + j);
    e->md.p_delta[j] = GET(ZB_V4_P_DELTA + j); e->md.actions[j] = GET(ZB_V4_ACTIONS + j);
  }
  e->md.commands[0] = GET(ZB_V4_COMMANDS); e->md.commands[1] = GET(ZB_V4_COMMANDS + 1);
  e->md.target_yaw = GET(ZB_V4_TARGET_YAW); e->md.interval_left = GET(ZB_V4_INTERVAL_LEFT);
  e->md.current_yaw = GET(ZB_V4_CURRENT_YAW);
  for (int f = 0; f < 2; ++f) {
    for (int a = 0; a < 3; ++a) e->md.feet_down_pos[f][a] = GET(ZB_V4_FEET_DOWN_POS + 3 * f + a);
    e->md.feet_step_len[f] = GET(ZB_V4_FEET_STEP_LEN + f);
    e->md.feet_f_last[f] = GET(ZB_V4_FEET_F_LAST + f);
    e->md.feet_air_cur[f] = GET(ZB_V4_FEET_AIR_CUR + f);
    e->md.feet_contact_cur[f] = GET(ZB_V4_FEET_CONTACT_CUR + f);
    e->md.feet_air_last[f] = GET(ZB_V4_FEET_AIR_LAST + f);
    e->md.feet_contact_last[f] = GET(ZB_V4_FEET_CONTACT_LAST + f);
    for (int h = 0; h < ZB_V4_HIST; ++h) e->md.feet_fz_hist[h][f] = GET(ZB_V4_FEET_FZ_HIST + 2 * h + f);
  }
  for (int h = 0; h < ZB_V4_HIST; ++h) e->md.undes_fmax_hist[h] = GET(ZB_V4_UNDES_FMAX_HIST + h);
  e->md.ep_len = (int32_t)lrint((double)st[(size_t)ZB_V4_EP_LEN * n + i]);
  for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) e->md.ep_sums[t] = GET(ZB_V4_EP_SUMS + t);
#undef GET
}

/* ========================================================================= manager-based env
 * zbot-6b-walking-m-v0: ManagerBasedRLEnv over Zbot6BFlatEnvCfg (zbotlab_env_cfg.py = "mgr.py",
 * config/zbot6b_manager/flat_env_cfg.py, mdp/rewards.py, terminations.py, curriculums.py) on
 * ZBOT_6S_V2_CFG (Isaac Lab root = the base link). Step order (ManagerBasedRLEnv.step): action
 * processing, 4 x (apply_action, physics, scene.update -> contact sensor with history 3 > 0 updated
 * every physics step), ep_len + 1, terminations, rewards, _reset_idx (curriculum, reset events,
 * managers), command compute, observations (additive noise). The counter-based draws are the
 * kernel's: reset pose 1..4, reset command 5..7, interval command 9..11, observation noise 16..37. */
#define M_DRAW_RESET_CMD 5
#define M_DRAW_CMD 9
#define M_DRAW_NOISE 16

/* UniformVelocityCommand._resample_command: lin x ~ U(ranges.lin_vel_x), lin y ~ U(ranges.lin_vel_y)
 * (s->yaw holds the lin_vel_y range for this task), ang z ~ U(0, 0), standing ~ U(0,1) <= rel */
static void m_resample(const zbo_sim* s, uint64_t h, int k0, real cmd[3], real* standing) {
  cmd[0] = draw(h, k0) * ((real)s->vel[1] - (real)s->vel[0]) + (real)s->vel[0];
  cmd[1] = draw(h, k0 + 1) * ((real)s->yaw[1] - (real)s->yaw[0]) + (real)s->yaw[0];
  cmd[2] = 0;
  *standing = draw(h, k0 + 2) <= (real)s->c.cmd_rel_standing ? 1 : 0;
}

/* the post-step articulation / sensor data the flat manager terms read */
typedef struct {
  real base_pos[3], base_quat[4];   /* root_link_pos_w / root_link_quat_w (= root_pos_w / root_quat_w) */
  real base_lin_vel[3];             /* root_link_lin_vel_w */
  real base_ang_vel[3];             /* root_link_ang_vel_w */
  real feet_pos[2][3], feet_quat[2][4], feet_vel[2][3]; /* body_link_pos/quat_w, body_lin_vel_w (COM) */
  real fz_hist[3][2], fn_hist[3][2];  /* net_forces_w_history[:, :, feet, 2] and its |F| */
  real air_last[2];                 /* last_air_time[feet] */
  real applied_torque[ND], joint_acc[ND];
  int32_t ep_len;
} m_post_t;

/* TerminationManager.compute + RewardManager.compute (weight x step_dt, cfg order). md: commands,
 * feet_down_pos / feet_step_len / feet_f_last (foot_step_length's env state), ep_sums (updated). */
static real m_mdp_eval(const zb_task_cfg* cfg, const m_post_t* P, mdp_t* md, const real act[ND], const real prev[ND],
                       real terms[ZB_M_NUM_REWARD_TERMS], int* low, int* close, int* tout) {
  const real step_dt = (real)(cfg->sim_dt * (float)cfg->decimation);
  /* terminations.py / Isaac Lab: time_out (ep_len >= max), root_height_below_minimum (0.2),
   * feet_close (terminations.py:186-191: |foot_0 - foot_1| < 0.12) */
  *tout = P->ep_len >= cfg->max_episode_length;
  *low = P->base_pos[2] < (real)cfg->termination_height;
  real fd[3];
  for (int a = 0; a < 3; ++a) fd[a] = P->feet_pos[0][a] - P->feet_pos[1][a];
  *close = sqrtr(v3_dot(fd, fd)) < (real)cfg->feet_close_min;
  const int terminated = *low || *close;
  real R[9];
  q_to_mat(P->base_quat, R);
  const real fwd[3] = {R[4], -R[1], 0}; /* GRAVITY_VEC_W x quat_apply(root_quat_w, y) (rewards.py:64-65) */
  { /* track_lin_vel_xy_yaw_frame_exp (rewards.py:289-301): yaw_quat + quat_apply_inverse */
    const real* q = P->base_quat;
    const double yaw = atan2(2.0 * ((double)q[0] * q[3] + (double)q[1] * q[2]),
                             1.0 - 2.0 * ((double)q[2] * q[2] + (double)q[3] * q[3]));
    const real c = (real)cos(yaw), sn = (real)sin(yaw);
    const real vx = c * P->base_lin_vel[0] + sn * P->base_lin_vel[1];
    const real vy = -sn * P->base_lin_vel[0] + c * P->base_lin_vel[1];
    const real ex = md->commands[0] - vx, ey = md->commands[1] - vy;
    terms[ZB_M_R_TRACK_LIN_VEL_XY] = (real)exp(-(double)(ex * ex + ey * ey) / 0.25);
    const real ez = md->commands[2] - P->base_ang_vel[2]; /* track_ang_vel_z_world_exp (303-312) */
    terms[ZB_M_R_TRACK_ANG_VEL_Z] = (real)exp(-(double)(ez * ez) / 0.25);
  }
  terms[ZB_M_R_TERMINATION] = (real)terminated;        /* is_terminated */
  real t2 = 0, a2 = 0, r2 = 0;
  for (int j = 0; j < ND; ++j) {
    t2 += P->applied_torque[j] * P->applied_torque[j]; /* joint_torques_l2 */
    a2 += P->joint_acc[j] * P->joint_acc[j];           /* joint_acc_l2 */
    r2 += (act[j] - prev[j]) * (act[j] - prev[j]);     /* action_rate_l2 */
  }
  terms[ZB_M_R_DOF_TORQUES] = t2;
  terms[ZB_M_R_DOF_ACC] = a2;
  terms[ZB_M_R_ACTION_RATE] = r2;
  { /* foot_step_length (rewards.py:44-104): touchdown = mean F_z over the history > 10 after < 10 */
    const real nrm = sqrtr(v3_dot(fwd, fwd)) + (real)1e-6;
    const real fh[3] = {fwd[0] / nrm, fwd[1] / nrm, fwd[2] / nrm};
    for (int f = 0; f < 2; ++f) {
      const real fz = (P->fz_hist[0][f] + P->fz_hist[1][f] + P->fz_hist[2][f]) / 3;
      if (fz > 10 && md->feet_f_last[f] < 10) {
        real dv[3];
        for (int a = 0; a < 3; ++a) dv[a] = P->feet_pos[f][a] - md->feet_down_pos[f][a];
        md->feet_step_len[f] = (real)fabs((double)v3_dot(dv, fh));
        for (int a = 0; a < 3; ++a) md->feet_down_pos[f][a] = P->feet_pos[f][a];
      }
      md->feet_f_last[f] = fz;
    }
    const real mn = md->feet_step_len[0] < md->feet_step_len[1] ? md->feet_step_len[0] : md->feet_step_len[1];
    terms[ZB_M_R_FOOT_STEP_LENGTH] = (real)tanh(15.0 * (double)mn);
  }
  real sd = 0, sf = 0, sl = 0;
  for (int f = 0; f < 2; ++f) {
    real Rf[9];
    q_to_mat(P->feet_quat[f], Rf);
    const real sg = f == 0 ? 1 : -1; /* foot_downward (106-121): feet axes (0, +-1, 0) vs world z */
    const real dz[3] = {sg * Rf[1], sg * Rf[4], sg * Rf[7] - 1};
    sd += sqrtr(v3_dot(dz, dz));
    const real dx[3] = {Rf[0] - fwd[0], Rf[3] - fwd[1], Rf[6] - fwd[2]}; /* foot_forward (123-142) */
    sf += sqrtr(v3_dot(dx, dx));
    real fm = P->fn_hist[0][f]; /* feet_slide (250-264): max |F| over the history > 1 */
    if (P->fn_hist[1][f] > fm) fm = P->fn_hist[1][f];
    if (P->fn_hist[2][f] > fm) fm = P->fn_hist[2][f];
    const real v2 = P->feet_vel[f][0] * P->feet_vel[f][0] + P->feet_vel[f][1] * P->feet_vel[f][1];
    sl += sqrtr(v2) * (fm > 1 ? 1 : 0);
  }
  terms[ZB_M_R_FOOT_DOWNWARD] = sd;
  terms[ZB_M_R_FOOT_FORWARD] = sf;
  terms[ZB_M_R_FEET_SLIDE] = sl;
  terms[ZB_M_R_AIR_TIME_BALANCE] = (real)fabs((double)(P->air_last[0] - P->air_last[1])); /* 241-248 */
  real rew = 0;
  for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) {
    const real v = terms[t] * (real)cfg->stage_scales[0][t] * step_dt;
    rew += v;
    md->ep_sums[t] += v;
  }
  return rew;
}

/* reset events (reset_base = reset_root_state_uniform, reset_robot_joints = defaults,
 * reset_my_data = feet data at the post-reset feet) and the managers' resets (actions,
 * episode sums, command resample + metrics, contact sensor). init: the construction-time reset. */
static void m_reset_env(const zbo_sim* s, uint64_t ctr, int i, env_t* e) {
  wc_invalidate(e->wc); /* the pose jumps: no warm start */
  const mdl_t* m = &s->m;
  const uint64_t h = env_hash(s->seed, ctr, i);
  mdp_t* md = &e->md;
  real pre[2][3];
  feet_world(m, &e->ph, pre);
  (void)reset_pose(m, &s->c, h, &e->ph);
  m_resample(s, h, M_DRAW_RESET_CMD, md->commands, &md->cmd_standing);
  md->interval_left = s->c.cmd_resample_s;
  md->metrics[0] = md->metrics[1] = 0;
  for (int j = 0; j < ND; ++j) md->actions[j] = 0;
  latch_feet(m, &s->c, pre, &e->ph, md->feet_down_pos);
  for (int f = 0; f < 2; ++f) {
    md->feet_f_last[f] = 0;
    md->feet_step_len[f] = 0;
    md->feet_air_cur[f] = md->feet_air_last[f] = 0;
    for (int h2 = 0; h2 < 3; ++h2) md->feet_fz_hist[h2][f] = md->feet_fn_hist[h2][f] = 0;
  }
  md->ep_len = 0;
  for (int t = 0; t < ZB_MAX_REWARD_TERMS; ++t) md->ep_sums[t] = 0;
}

/* policy group (mgr.py:139-161): root_quat_w, generated_commands, joint_pos_rel, joint_vel_rel
 * (Isaac Lab joint order), last_action; additive U(-n, n) on quat / joint pos / joint vel */
static void m_write_obs(const zbo_sim* s, const env_t* e, uint64_t h, float* obs) {
  const mdl_t* m = &s->m;
  const zb_task_cfg* c = &s->c;
  kin_t k;
  fk(m, &e->ph, &k);
  real p[3], q[4];
  link_pose(m, &k, m->base_link, p, q);
  const real cor = c->obs_corruption ? 1 : 0;
#define NOISE(kk, nn) (cor * (draw(h, M_DRAW_NOISE + (kk)) * (2 * (real)(nn)) - (real)(nn)))
  for (int a = 0; a < 4; ++a) obs[a] = (float)(q[a] + NOISE(a, c->obs_noise[0]));
  for (int a = 0; a < 3; ++a) obs[4 + a] = (float)e->md.commands[a];
  for (int j = 0; j < ND; ++j) {
    const int ai = m->api_index[j];
    obs[7 + ai] = (float)(m->api_sign[j] * (e->ph.jq[j] - m->jq0[j]) + NOISE(4 + ai, c->obs_noise[1]));
    obs[13 + ai] = (float)(m->api_sign[j] * e->ph.jqd[j] + NOISE(10 + ai, c->obs_noise[2]));
  }
#undef NOISE
  for (int a = 0; a < ND; ++a) obs[19 + a] = (float)e->md.actions[a];
}

/* UniformVelocityCommand._update_metrics with root_lin_vel_b / root_ang_vel_b (the base link's
 * COM velocity and angular velocity in its frame), then the timer / resample / standing zeroing */
static void m_command_compute(const zbo_sim* s, uint64_t h, env_t* e, const real vb[3], const real wb[3]) {
  mdp_t* md = &e->md;
  const zb_task_cfg* c = &s->c;
  const real step_dt = (real)(c->sim_dt * (float)c->decimation);
  const real max_steps = (real)c->cmd_resample_s / step_dt;
  const real ex = md->commands[0] - vb[0], ey = md->commands[1] - vb[1];
  md->metrics[0] += sqrtr(ex * ex + ey * ey) / max_steps;
  md->metrics[1] += (real)fabs((double)(md->commands[2] - wb[2])) / max_steps;
  md->interval_left -= step_dt;
  if (md->interval_left <= 0) {
    m_resample(s, h, M_DRAW_CMD, md->commands, &md->cmd_standing);
    md->interval_left = c->cmd_resample_s;
  }
  if (md->cmd_standing > (real)0.5) md->commands[0] = md->commands[1] = md->commands[2] = 0;
}

static real m_step_env(const zbo_sim* s, uint64_t ctr, int i, env_t* e, const float* action, float* obs, int* low,
                       int* close, int* tout, real acc[ZB_MAX_REWARD_TERMS], double met[2]) {
  const mdl_t* m = &s->m;
  const zb_task_cfg* cfg = &s->c;
  mdp_t* md = &e->md;
  /* RelativeJointPositionAction.process_actions: raw * scale (zero offset), clipped; Isaac Lab
   * joint order -> chain joints */
  real act[ND], prev[ND], delta[ND];
  for (int a = 0; a < ND; ++a) { act[a] = (real)action[a]; prev[a] = md->actions[a]; }
  for (int j = 0; j < ND; ++j)
    delta[j] = m->api_sign[j] * clampr(act[m->api_index[j]] * (real)cfg->action_scale, -(real)cfg->action_clip,
                                       (real)cfg->action_clip);
  substep_out_t so;
  real jqd_prev[ND];
  clist_t wl;
  wc_warm_list(e->wc, &wl);
  for (int k = 0; k < cfg->decimation; ++k) {
    real target[ND];
    for (int j = 0; j < ND; ++j) target[j] = e->ph.jq[j] + delta[j]; /* apply_actions: q + delta */
    if (k == cfg->decimation - 1)
      for (int j = 0; j < ND; ++j) jqd_prev[j] = e->ph.jqd[j];
    substep(m, cfg, &e->ph, target, md->mu, md->mu_d, &wl, &so);
    /* ContactSensor.update (every physics step): history shift, air time with elapsed sim_dt */
    for (int f = 0; f < 2; ++f) {
      const real* F = so.net_force[m->foot_links[f]];
      const real fn = sqrtr(v3_dot(F, F));
      md->feet_fz_hist[2][f] = md->feet_fz_hist[1][f];
      md->feet_fz_hist[1][f] = md->feet_fz_hist[0][f];
      md->feet_fz_hist[0][f] = F[2];
      md->feet_fn_hist[2][f] = md->feet_fn_hist[1][f];
      md->feet_fn_hist[1][f] = md->feet_fn_hist[0][f];
      md->feet_fn_hist[0][f] = fn;
      const int c = fn > (real)cfg->contact_force_threshold;
      if (md->feet_air_cur[f] > 0 && c) md->feet_air_last[f] = md->feet_air_cur[f] + (real)cfg->sim_dt;
      md->feet_air_cur[f] = c ? 0 : md->feet_air_cur[f] + (real)cfg->sim_dt;
    }
  }
  wc_store(&wl, e->wc);
  md->ep_len += 1;
  m_post_t P;
  real vcom[3];
  {
    kin_t k;
    fk(m, &e->ph, &k);
    real V[NB][6];
    body_vel(&k, &e->ph, V);
    const int B = m->base_link, bb = m->link_body[B];
    link_pose(m, &k, B, P.base_pos, P.base_quat);
    real x[3];
    m3_v(k.R[bb], m->link_pos[B], x);
    for (int a = 0; a < 3; ++a) x[a] += k.p[bb][a];
    point_vel(V[bb], x, P.base_lin_vel);
    m3_v(k.R[bb], m->link_com[B], x);
    for (int a = 0; a < 3; ++a) x[a] += k.p[bb][a];
    point_vel(V[bb], x, vcom);
    for (int a = 0; a < 3; ++a) { P.base_ang_vel[a] = V[bb][a]; P.base_pos[a] += e->ph.root_pos[a]; }
    for (int f = 0; f < 2; ++f) {
      const int l = m->foot_links[f], b = m->link_body[l];
      link_pose(m, &k, l, P.feet_pos[f], P.feet_quat[f]);
      for (int a = 0; a < 3; ++a) P.feet_pos[f][a] += e->ph.root_pos[a];
      real c[3];
      m3_v(k.R[b], m->link_com[l], c);
      for (int a = 0; a < 3; ++a) c[a] += k.p[b][a];
      point_vel(V[b], c, P.feet_vel[f]);
    }
  }
  for (int j = 0; j < ND; ++j) {
    P.applied_torque[j] = so.applied_torque[j];
    P.joint_acc[j] = (e->ph.jqd[j] - jqd_prev[j]) / (real)cfg->sim_dt;
  }
  for (int h = 0; h < 3; ++h)
    for (int f = 0; f < 2; ++f) { P.fz_hist[h][f] = md->feet_fz_hist[h][f]; P.fn_hist[h][f] = md->feet_fn_hist[h][f]; }
  P.air_last[0] = md->feet_air_last[0];
  P.air_last[1] = md->feet_air_last[1];
  P.ep_len = md->ep_len;
  for (int a = 0; a < ND; ++a) md->actions[a] = act[a];
  real terms[ZB_M_NUM_REWARD_TERMS];
  const real rew = m_mdp_eval(cfg, &P, md, act, prev, terms, low, close, tout);
  const uint64_t h = env_hash(s->seed, ctr, i);
  real vb[3] = {0, 0, 0}, wb[3] = {0, 0, 0};
  if (*low || *close || *tout) {
    for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) acc[t] += md->ep_sums[t];
    met[0] += md->metrics[0];
    met[1] += md->metrics[1];
    m_reset_env(s, ctr, i, e);
  } else {
    real Rb[9];
    q_to_mat(P.base_quat, Rb);
    for (int a = 0; a < 3; ++a) {
      vb[a] = Rb[a] * vcom[0] + Rb[3 + a] * vcom[1] + Rb[6 + a] * vcom[2];
      wb[a] = Rb[a] * P.base_ang_vel[0] + Rb[3 + a] * P.base_ang_vel[1] + Rb[6 + a] * P.base_ang_vel[2];
    }
  }
  m_command_compute(s, h, e, vb, wb);
  m_write_obs(s, e, h, obs);
  return rew;
}

/* a reset env's command redrawn after lin_vel_cmd_levels widened the ranges in the same call
 * (the reference's curriculum runs before the command manager's reset); velocity 0 after reset */
static void m_fixup_env(const zbo_sim* s, uint64_t ctr, int i, env_t* e, float* obs) {
  mdp_t* md = &e->md;
  const uint64_t h = env_hash(s->seed, ctr, i);
  m_resample(s, h, M_DRAW_RESET_CMD, md->commands, &md->cmd_standing);
  md->metrics[0] = md->metrics[1] = 0;
  md->interval_left = s->c.cmd_resample_s;
  const real zero[3] = {0, 0, 0};
  m_command_compute(s, h, e, zero, zero);
  for (int a = 0; a < 3; ++a) obs[4 + a] = (float)md->commands[a];
}

static void m_pack_env(const env_t* e, float* st, int n, int i) {
#define PUT(off, val) st[(size_t)(off) * n + i] = (float)(val)
  for (int a = 0; a < 3; ++a) { PUT(ZB_S_ROOT_POS + a, e->ph.root_pos[a]); PUT(ZB_S_ROOT_LINVEL + a, e->ph.root_linvel[a]); PUT(ZB_S_ROOT_ANGVEL + a, e->ph.root_angvel[a]); }
  for (int a = 0; a < 4; ++a) PUT(ZB_S_ROOT_QUAT + a, e->ph.root_quat[a]);
  for (int j = 0; j < ND; ++j) { PUT(ZB_S_JOINT_POS + j, e->ph.jq[j]); PUT(ZB_S_JOINT_VEL + j, e->ph.jqd[j]); PUT(ZB_M_ACTIONS + j, e->md.actions[j]); }
  for (int a = 0; a < 3; ++a) PUT(ZB_M_COMMANDS + a, e->md.commands[a]);
  PUT(ZB_M_CMD_TIME_LEFT, e->md.interval_left);
  PUT(ZB_M_CMD_STANDING, e->md.cmd_standing);
  PUT(ZB_M_METRICS, e->md.metrics[0]);
  PUT(ZB_M_METRICS + 1, e->md.metrics[1]);
  for (int f = 0; f < 2; ++f) {
    for (int a = 0; a < 3; ++a) PUT(ZB_M_FEET_DOWN_POS + 3 * f + a, e->md.feet_down_pos[f][a]);
    PUT(ZB_M_FEET_STEP_LEN + f, e->md.feet_step_len[f]);
    PUT(ZB_M_FEET_F_LAST + f, e->md.feet_f_last[f]);
    PUT(ZB_M_FEET_AIR_CUR + f, e->md.feet_air_cur[f]);
    PUT(ZB_M_FEET_AIR_LAST + f, e->md.feet_air_last[f]);
    for (int h = 0; h < 3; ++h) { PUT(ZB_M_FEET_FZ_HIST + 2 * h + f, e->md.feet_fz_hist[h][f]); PUT(ZB_M_FEET_FN_HIST + 2 * h + f, e->md.feet_fn_hist[h][f]); }
  }
  PUT(ZB_M_EP_LEN, e->md.ep_len);
  for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) PUT(ZB_M_EP_SUMS + t, e->md.ep_sums[t]);
  for (int l = 0; l < NL; ++l) { PUT(ZB_M_LINK_MU + l, e->md.mu[l]); PUT(ZB_M_LINK_MU_D + l, e->md.mu_d[l]); }
#undef PUT
}

static void m_unpack_env(env_t* e, const float* st, int n, int i) {
#define GET(off) ((real)st[(size_t)(off) * n + i])
  for (int a = 0; a < 3; ++a) { e->ph.root_pos[a] = GET(ZB_S_ROOT_POS + a); e->ph.root_linvel[a] = GET(ZB_S_ROOT_LINVEL + a); e->ph.root_angvel[a] = GET(ZB_S_ROOT_ANGVEL + a); }
  for (int a = 0; a < 4; ++a) e->ph.root_quat[a] = GET(ZB_S_ROOT_QUAT + a);
  for (int j = 0; j < ND; ++j) { e->ph.jq[j] = GET(ZB_S_JOINT_POS + j); e->ph.jqd[j] = GET(ZB_S_JOINT_VEL + j); e->md.actions[j] = GET(ZB_M_ACTIONS + j); }
  for (int a = 0; a < 3; ++a) e->md.commands[a] = GET(ZB_M_COMMANDS + a);
  e->md.interval_left = GET(ZB_M_CMD_TIME_LEFT);
  e->md.cmd_standing = GET(ZB_M_CMD_STANDING);
  e->md.metrics[0] = GET(ZB_M_METRICS);
  e->md.metrics[1] = GET(ZB_M_METRICS + 1);
  for (int f = 0; f < 2; ++f) {
    for (int a = 0; a < 3; ++a) e->md.feet_down_pos[f][a] = GET(ZB_M_FEET_DOWN_POS + 3 * f + a);
    e->md.feet_step_len[f] = GET(ZB_M_FEET_STEP_LEN + f);
    e->md.feet_f_last[f] = GET(ZB_M_FEET_F_LAST + f);
    e->md.feet_air_cur[f] = GET(ZB_M_FEET_AIR_CUR + f);
    e->md.feet_air_last[f] = GET(ZB_M_FEET_AIR_LAST + f);
    for (int h = 0; h < 3; ++h) { e->md.feet_fz_hist[h][f] = GET(ZB_M_FEET_FZ_HIST + 2 * h + f); e->md.feet_fn_hist[h][f] = GET(ZB_M_FEET_FN_HIST + 2 * h + f); }
  }
  e->md.ep_len = (int32_t)lrint((double)st[(size_t)ZB_M_EP_LEN * n + i]);
  for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) e->md.ep_sums[t] = GET(ZB_M_EP_SUMS + t);
  for (int l = 0; l < NL; ++l) { e->md.mu[l] = GET(ZB_M_LINK_MU + l); e->md.mu_d[l] = GET(ZB_M_LINK_MU_D + l); }
#undef GET
}

/* lin_vel_cmd_levels (curriculums.py:57-83) on the mean episodic tracking reward / 20 s of the reset
 * envs; vel = ranges.lin_vel_x, yaw = ranges.lin_vel_y. Returns 1 when it widened the ranges. */
static int m_lin_vel_cmd_levels(const zb_task_cfg* c, uint64_t steps, float reward, float vel[2], float yaw[2]) {
  if (c->range_period_steps <= 0 || steps % (uint64_t)c->range_period_steps != 0) return 0;
  if (!(reward > c->stage_scales[0][ZB_M_R_TRACK_LIN_VEL_XY] * c->range_threshold)) return 0;
  vel[0] = (float)clampr(vel[0] - c->range_delta, c->range_limit_vel[0], c->range_limit_vel[1]);
  vel[1] = (float)clampr(vel[1] + c->range_delta, c->range_limit_vel[0], c->range_limit_vel[1]);
  yaw[0] = (float)clampr(yaw[0] - c->range_delta, c->range_limit_yaw[0], c->range_limit_yaw[1]);
  yaw[1] = (float)clampr(yaw[1] + c->range_delta, c->range_limit_yaw[0], c->range_limit_yaw[1]);
  return 1;
}

/* ========================================================================= call epilogue
 * Mirror of the kernel's zb_finalize_kernel: episode log (means over reset envs; walking divides
 * by the 20 s episode, the other tasks already divided per env), curriculum log entries (pre-event
 * values), v4 range-curriculum buffers, my_curriculum, range_curriculum, full-reset ep_len draw. */
static void curriculum_events(zbo_sim* s, int run_my, int run_range);

static void finish_call(zbo_sim* s, int nres, const double* acc, double ep_s, int nterm, int ntout, int reset_counts,
                        int full) {
  const uint64_t ctr = s->call_counter;
  const zb_task_cfg* c = &s->c;
  if (nres > 0) {
    float v[ZB_LOG_LEN];
    for (int t = 0; t < ZB_MAX_REWARD_TERMS; ++t) v[t] = (float)(acc[t] / nres / ep_s);
    v[16] = (float)s->stage;
    v[17] = s->vel[0];
    v[18] = s->vel[1];
    v[19] = s->yaw[0];
    if (c->task == ZB_TASK_MANAGER_V0) {
      /* lin_vel_cmd_levels (curriculums.py:57-83), first in _reset_idx: on calls where
       * common_step_counter % max_episode_length == 0, widen the x / y ranges by +-0.1 (clamped to
       * limit_ranges) when mean(episode sums of track_lin_vel_xy_exp) / 20 s > 0.8 x weight */
      s->changed = m_lin_vel_cmd_levels(c, s->steps, v[ZB_M_R_TRACK_LIN_VEL_XY], s->vel, s->yaw);
      v[16] = s->vel[1];                       /* Curriculum/lin_vel_cmd_levels */
      v[17] = (float)(s->met_acc[0] / nres);   /* Metrics/base_velocity/error_vel_xy */
      v[18] = (float)(s->met_acc[1] / nres);   /* Metrics/base_velocity/error_vel_yaw */
      v[19] = 0;
    }
    for (int t = 0; t < ZB_LOG_LEN; ++t) s->log_means[t] = v[t];
    s->log_counts[0] = reset_counts ? 0 : nterm;
    s->log_counts[1] = reset_counts ? 0 : ntout;
    s->log_counts[2] = reset_counts ? 0 : s->nclose;
    s->log_counts[3] = 0;
    if (c->task == ZB_TASK_WALKING_V4) {
      s->ring_vel[s->ring_head] = v[ZB_V4_R_TRACK_LIN_VEL_X];
      s->ring_yaw[s->ring_head] = v[ZB_V4_R_TRACK_HEADING_YAW];
      s->ring_head = (s->ring_head + 1) % ZB_V4_RING;
      if (s->ring_n < ZB_V4_RING) s->ring_n++;
    }
    curriculum_events(s, 1, 1);
  }
  s->call_counter++;
  if (full && c->task != ZB_TASK_MANAGER_V0) /* ManagerBasedRLEnv has no full-reset draw */
    for (int e = 0; e < s->n; ++e) /* episode_length_buf ~ U{0..max_episode_length-1} (v2.py:418-422) */
      s->env[e].md.ep_len = (int32_t)(env_hash(s->seed, ctr, e) % (uint64_t)c->max_episode_length);
}

/* reset-mode curriculum events in EventCfg order: my_curriculum (one stage per call), then
 * range_curriculum (v4) on the buffered per-call tracking rewards */
static void curriculum_events(zbo_sim* s, int run_my, int run_range) {
  const zb_task_cfg* c = &s->c;
  {
    if (run_my && s->stage + 1 < c->num_stages && s->steps >= (uint64_t)c->stage_steps[s->stage + 1]) {
      s->stage++;
      s->prob_pos = c->stage_prob_pos[s->stage];
    }
    /* range_curriculum (v4.py:201-265) */
    if (run_range && c->task == ZB_TASK_WALKING_V4 && s->ring_n >= c->range_min_buffer && c->range_period_steps > 0 &&
        s->steps >= (uint64_t)c->range_start_steps && s->steps % (uint64_t)c->range_period_steps == 0) {
      float mv = 0, my = 0;
      for (int k = 0; k < s->ring_n; ++k) { mv += s->ring_vel[k]; my += s->ring_yaw[k]; }
      mv /= (float)s->ring_n;
      my /= (float)s->ring_n;
      if (mv > c->stage_scales[s->stage][ZB_V4_R_TRACK_LIN_VEL_X] * c->range_threshold) {
        s->vel[0] = (float)clampr(s->vel[0] - c->range_delta, c->range_limit_vel[0], c->range_limit_vel[1]);
        s->vel[1] = (float)clampr(s->vel[1] + c->range_delta, c->range_limit_vel[0], c->range_limit_vel[1]);
      }
      if (my > c->stage_scales[s->stage][ZB_V4_R_TRACK_HEADING_YAW] * c->range_threshold) {
        s->yaw[0] = (float)clampr(s->yaw[0] - c->range_delta, c->range_limit_yaw[0], c->range_limit_yaw[1]);
        s->yaw[1] = (float)clampr(s->yaw[1] + c->range_delta, c->range_limit_yaw[0], c->range_limit_yaw[1]);
      }
    }
  }
}

/* ========================================================================= public API */
#ifdef _OPENMP
#include <omp.h>
#endif

zbo_sim* zbo_create(const zb_model* model, const zb_task_cfg* cfg, int num_envs, uint64_t seed) {
  zbo_sim* s = (zbo_sim*)calloc(1, sizeof(zbo_sim));
  load_mdl(model, &s->m);
  s->c = *cfg;
  s->n = num_envs;
  s->seed = seed;
  s->vel[0] = cfg->cmd_vel_range[0]; s->vel[1] = cfg->cmd_vel_range[1];
  s->yaw[0] = cfg->cmd_yaw_range[0]; s->yaw[1] = cfg->cmd_yaw_range[1];
  s->prob_pos = cfg->stage_prob_pos[0];
  s->env = (env_t*)calloc((size_t)num_envs, sizeof(env_t));
  s->act = (int32_t*)calloc((size_t)num_envs * 2, sizeof(int32_t));
  for (int i = 0; i < num_envs; ++i) {
    memset(&s->env[i], 0, sizeof(env_t));
    wc_invalidate(s->env[i].wc);
    phys_default(&s->m, &s->env[i].ph); /* the spawn pose: what the construction-time reset's latch reads */
    if (cfg->task == ZB_TASK_STANDUP_V0) {
      for (int l = 0; l < NL; ++l) { s->env[i].md.mu[l] = cfg->friction; s->env[i].md.mu_d[l] = cfg->friction_dynamic; }
      su_reset_env(&s->m, cfg, seed, 0, i, &s->env[i]); /* construction draws at RNG position 0 */
    } else if (cfg->task == ZB_TASK_WALKING_V4) {
      v4_reset_env(s, 0, i, &s->env[i], 1);
    } else if (cfg->task == ZB_TASK_MANAGER_V0) {
      for (int l = 0; l < NL; ++l) { s->env[i].md.mu[l] = cfg->friction; s->env[i].md.mu_d[l] = cfg->friction_dynamic; }
      m_reset_env(s, 0, i, &s->env[i]);
    } else {
      reset_env(&s->m, cfg, &s->env[i]);
    }
  }
  if (cfg->task != ZB_TASK_WALKING_V2) s->call_counter = 1;
  return s;
}

void zbo_destroy(zbo_sim* s) {
  if (!s) return;
  free(s->env);
  free(s->act);
  free(s);
}

int zbo_set_threads(int n) {
#ifdef _OPENMP
  if (n > 0) omp_set_num_threads(n);
  return omp_get_max_threads();
#else
  (void)n;
  return 1;
#endif
}

int zbo_reset(zbo_sim* s, const int32_t* env_ids, int n) {
  const int all = env_ids == NULL || n == s->n;
  const int cnt = env_ids ? n : s->n;
  const uint64_t ctr = s->call_counter;
  const real step_dt = (real)(s->c.sim_dt * (float)s->c.decimation);
  double acc[ZB_MAX_REWARD_TERMS];
  for (int t = 0; t < ZB_MAX_REWARD_TERMS; ++t) acc[t] = 0;
  s->met_acc[0] = s->met_acc[1] = 0;
  s->nclose = 0;
  s->changed = 0;
  for (int i = 0; i < cnt; ++i) {
    const int e = env_ids ? env_ids[i] : i;
    env_t* en = &s->env[e];
    if (s->c.task == ZB_TASK_MANAGER_V0) {
      for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) acc[t] += en->md.ep_sums[t];
      s->met_acc[0] += en->md.metrics[0];
      s->met_acc[1] += en->md.metrics[1];
      m_reset_env(s, ctr, e, en);
    } else if (s->c.task == ZB_TASK_WALKING_V2) {
      for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) acc[t] += en->md.ep_sums[t];
      reset_env(&s->m, &s->c, en);
    } else {
      real dur = (real)en->md.ep_len * step_dt;
      if (dur < step_dt) dur = step_dt;
      for (int t = 0; t < ZB_MAX_REWARD_TERMS; ++t) acc[t] += en->md.ep_sums[t] / dur;
      if (s->c.task == ZB_TASK_STANDUP_V0) su_reset_env(&s->m, &s->c, s->seed, ctr, e, en);
      else v4_reset_env(s, ctr, e, en, 0);
    }
  }
  const int per_episode = s->c.task == ZB_TASK_WALKING_V2 || s->c.task == ZB_TASK_MANAGER_V0;
  const double ep_s = per_episode ? (double)(s->c.sim_dt * (float)s->c.decimation * (float)s->c.max_episode_length) : 1.0;
  finish_call(s, cnt, acc, ep_s, 0, 0, 1, all);
  return 0;
}

int zbo_observe(zbo_sim* s, float* obs) {
  for (int e = 0; e < s->n; ++e) {
    if (s->c.task == ZB_TASK_STANDUP_V0) su_write_obs(&s->m, &s->env[e], obs + (size_t)e * ZB_SU_OBS_DIM);
    else if (s->c.task == ZB_TASK_WALKING_V4) v4_write_obs(&s->m, &s->env[e], obs + (size_t)e * ZB_V4_OBS_DIM);
    else if (s->c.task == ZB_TASK_MANAGER_V0)
      m_write_obs(s, &s->env[e], env_hash(s->seed, s->call_counter, e), obs + (size_t)e * ZB_M_OBS_DIM);
    else write_obs(&s->m, &s->env[e], obs + (size_t)e * ZB_OBS_DIM);
  }
  return 0;
}

/* full walking-v2 policy step for env e; returns reward, sets flags; accumulates the log */
static real step_env(const mdl_t* m, const zb_task_cfg* cfg, env_t* e, const float* action, float* obs,
                     int* died, int* tout, real acc[ZB_MAX_REWARD_TERMS]) {
  mdp_t* md = &e->md;
  /* _pre_physics_step (v2.py:276-287) */
  real act[ND], prev[ND], target[ND];
  for (int j = 0; j < ND; ++j) {
    prev[j] = md->actions[j];
    act[j] = (real)tanh((double)action[j]);
    real pd = md->p_delta[j] + (real)PI_R * act[j] * cfg->joint_speed_limit * (cfg->sim_dt * cfg->decimation);
    pd = clampr(pd, -(real)PI_R, (real)PI_R);
    md->p_delta[j] = pd;
    target[j] = pd + m->jq0[j];
  }
  /* the previous step's _get_observations cache (one-step lag) */
  obs_cache_t pre;
  cache_from_phys(m, &e->ph, &pre);
  /* physics */
  substep_out_t so;
  clist_t wl;
  wc_warm_list(e->wc, &wl); /* the first substep's warm start: the cache */
  for (int k = 0; k < cfg->decimation; ++k) {
    substep(m, cfg, &e->ph, target, NULL, NULL, &wl, &so);
    sensor_update(m, cfg, md, so.net_force);
  }
  wc_store(&wl, e->wc);
  md->ep_len += 1;
  /* post-step reads */
  post_t ps;
  {
    kin_t k;
    fk(m, &e->ph, &k);
    real V[NB][6];
    body_vel(&k, &e->ph, V);
    for (int f = 0; f < 2; ++f) {
      int l = m->foot_links[f], b = m->link_body[l];
      real c[3];
      m3_v(k.R[b], m->link_com[l], c);
      for (int a = 0; a < 3; ++a) c[a] += k.p[b][a];
      point_vel(V[b], c, ps.feet_vel[f]);
    }
  }
  for (int j = 0; j < ND; ++j) { ps.jq[j] = e->ph.jq[j]; ps.jqd[j] = e->ph.jqd[j]; ps.applied_torque[j] = so.applied_torque[j]; }
  for (int h = 0; h < ZB_HIST; ++h) {
    ps.feet_fz_hist[h][0] = md->feet_fz_hist[h][0];
    ps.feet_fz_hist[h][1] = md->feet_fz_hist[h][1];
    ps.undes_fmax_hist[h] = md->undes_fmax_hist[h];
  }
  ps.feet_air_last[0] = md->feet_air_last[0];
  ps.feet_air_last[1] = md->feet_air_last[1];
  ps.ep_len = md->ep_len;
  ps.origin_y = 0;
  real terms[ZB_NUM_REWARD_TERMS];
  for (int j = 0; j < ND; ++j) md->actions[j] = act[j];
  real rew = mdp_eval(cfg, m->jq0, &pre, &ps, md, act, prev, terms, died, tout);
  if (*died || *tout) {
    for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) acc[t] += md->ep_sums[t];
    reset_env(m, cfg, e);
  }
  write_obs(m, e, obs);
  return rew;
}

int zbo_step(zbo_sim* s, const float* actions, float* obs, float* reward, uint8_t* terminated, uint8_t* truncated) {
  double acc[ZB_MAX_REWARD_TERMS];
  for (int t = 0; t < ZB_MAX_REWARD_TERMS; ++t) acc[t] = 0;
  int nreset = 0, nterm = 0, ntout = 0;
  const uint64_t ctr = s->call_counter;
  const int stage = s->stage;
  const int task = s->c.task;
  const int od = task == ZB_TASK_STANDUP_V0 ? ZB_SU_OBS_DIM : task == ZB_TASK_WALKING_V4 ? ZB_V4_OBS_DIM
               : task == ZB_TASK_MANAGER_V0 ? ZB_M_OBS_DIM : ZB_OBS_DIM;
  s->steps++; /* DirectRLEnv / ManagerBasedRLEnv.step: common_step_counter += 1 before dones / rewards / resets */
  s->met_acc[0] = s->met_acc[1] = 0;
  s->nclose = 0;
  s->changed = 0;
  int nclose = 0;
  double met0 = 0, met1 = 0;
#pragma omp parallel
  {
    real acc_l[ZB_MAX_REWARD_TERMS];
    double met_l[2] = {0, 0};
    int nr = 0, nt = 0, no = 0, nc = 0;
    for (int t = 0; t < ZB_MAX_REWARD_TERMS; ++t) acc_l[t] = 0;
#pragma omp for schedule(static)
    for (int e = 0; e < s->n; ++e) {
      int died = 0, tout = 0, close = 0;
      const float* a = actions + (size_t)e * ZB_ACT_DIM;
      float* o = obs + (size_t)e * od;
      real r;
      t_act = s->act + 2 * (size_t)e;
      if (task == ZB_TASK_STANDUP_V0) r = su_step_env(&s->m, &s->c, stage, s->seed, ctr, e, &s->env[e], a, o, &died, &tout, acc_l);
      else if (task == ZB_TASK_WALKING_V4) r = v4_step_env(s, stage, ctr, e, &s->env[e], a, o, &died, &tout, acc_l);
      else if (task == ZB_TASK_MANAGER_V0) r = m_step_env(s, ctr, e, &s->env[e], a, o, &died, &close, &tout, acc_l, met_l);
      else r = step_env(&s->m, &s->c, &s->env[e], a, o, &died, &tout, acc_l);
      t_act = NULL;
      reward[e] = (float)r;
      /* manager: terminated = base_height | feet_close; the log counts each term */
      terminated[e] = (uint8_t)(died || close);
      truncated[e] = (uint8_t)tout;
      nr += died || close || tout; nt += died; no += tout; nc += close;
    }
#pragma omp critical
    {
      for (int t = 0; t < ZB_MAX_REWARD_TERMS; ++t) acc[t] += acc_l[t];
      nreset += nr; nterm += nt; ntout += no; nclose += nc;
      met0 += met_l[0]; met1 += met_l[1];
    }
  }
  s->met_acc[0] = met0;
  s->met_acc[1] = met1;
  s->nclose = nclose;
  const int per_episode = task == ZB_TASK_WALKING_V2 || task == ZB_TASK_MANAGER_V0;
  const double ep_s = per_episode ? (double)(s->c.sim_dt * (float)s->c.decimation * (float)s->c.max_episode_length) : 1.0;
  finish_call(s, nreset, acc, ep_s, nterm, ntout, 0, nreset == s->n);
  if (task == ZB_TASK_MANAGER_V0 && s->changed)
    for (int e = 0; e < s->n; ++e)
      if (terminated[e] || truncated[e]) m_fixup_env(s, ctr, e, &s->env[e], obs + (size_t)e * od);
  return 0;
}

/* test hook: per env [loaded ground contacts, loaded self contacts] (lambda_n > 0 after the
 * solve) summed over the substeps of the zbo_step calls since the last clear */
int zbo_contact_activity(zbo_sim* s, int32_t* out, int clear) {
  memcpy(out, s->act, (size_t)s->n * 2 * sizeof(int32_t));
  if (clear) memset(s->act, 0, (size_t)s->n * 2 * sizeof(int32_t));
  return 0;
}

int zbo_read_log(zbo_sim* s, float* term_means, int32_t* counts) {
  for (int t = 0; t < ZB_LOG_LEN; ++t) term_means[t] = s->log_means[t];
  for (int k = 0; k < ZB_LOG_COUNTS; ++k) counts[k] = s->log_counts[k];
  return 0;
}

/* state <-> SoA [ZB_STATE_DIM][N] */
static void pack_env(const env_t* e, float* st, int n, int i) {
#define PUT(off, val) st[(size_t)(off) * n + i] = (float)(val)
  for (int a = 0; a < 3; ++a) { PUT(ZB_S_ROOT_POS + a, e->ph.root_pos[a]); PUT(ZB_S_ROOT_LINVEL + a, e->ph.root_linvel[a]); PUT(ZB_S_ROOT_ANGVEL + a, e->ph.root_angvel[a]); }
  for (int a = 0; a < 4; ++a) PUT(ZB_S_ROOT_QUAT + a, e->ph.root_quat[a]);
  for (int j = 0; j < ND; ++j) {
    PUT(ZB_S_JOINT_POS + j, e->ph.jq[j]); PUT(ZB_S_JOINT_VEL + j, e->ph.jqd[j]);
    PUT(ZB_S_P_DELTA + j, e->md.p_delta[j]); PUT(ZB_S_ACTIONS + j, e->md.actions[j]);
  }
  for (int f = 0; f < 2; ++f) {
    for (int a = 0; a < 3; ++a) PUT(ZB_S_FEET_DOWN_POS + 3 * f + a, e->md.feet_down_pos[f][a]);
    PUT(ZB_S_FEET_STEP_LEN + f, e->md.feet_step_len[f]);
    PUT(ZB_S_FEET_F_LAST + f, e->md.feet_f_last[f]);
    PUT(ZB_S_FEET_AIR_CUR + f, e->md.feet_air_cur[f]);
    PUT(ZB_S_FEET_AIR_LAST + f, e->md.feet_air_last[f]);
    PUT(ZB_S_FEET_CONTACT_CUR + f, e->md.feet_contact_cur[f]);
  }
  PUT(ZB_S_HEADING_SUM, e->md.heading_sum);
  PUT(ZB_S_Y_ERR_SUM, e->md.yerr_sum);
  PUT(ZB_S_FEET_FORCE_SUM, e->md.force_sum);
  for (int h = 0; h < ZB_HIST; ++h) {
    PUT(ZB_S_FEET_FZ_HIST + 2 * h, e->md.feet_fz_hist[h][0]);
    PUT(ZB_S_FEET_FZ_HIST + 2 * h + 1, e->md.feet_fz_hist[h][1]);
    PUT(ZB_S_UNDES_FMAX_HIST + h, e->md.undes_fmax_hist[h]);
  }
  PUT(ZB_S_EP_LEN, e->md.ep_len);
  for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) PUT(ZB_S_EP_SUMS + t, e->md.ep_sums[t]);
#undef PUT
}
static void unpack_env(env_t* e, const float* st, int n, int i) {
#define GET(off) ((real)st[(size_t)(off) * n + i])
  for (int a = 0; a < 3; ++a) { e->ph.root_pos[a] = GET(ZB_S_ROOT_POS + a); e->ph.root_linvel[a] = GET(ZB_S_ROOT_LINVEL + a); e->ph.root_angvel[a] = GET(ZB_S_ROOT_ANGVEL + a); }
  for (int a = 0; a < 4; ++a) e->ph.root_quat[a] = GET(ZB_S_ROOT_QUAT + a);
  for (int j = 0; j < ND; ++j) {
    e->ph.jq[j] = GET(ZB_S_JOINT_POS + j); e->ph.jqd[j] = GET(ZB_S_JOINT_VEL + j);
    e->md.p_delta[j] = GET(ZB_S_P_DELTA + j); e->md.actions[j] = GET(ZB_S_ACTIONS + j);
  }
  for (int f = 0; f < 2; ++f) {
    for (int a = 0; a < 3; ++a) e->md.feet_down_pos[f][a] = GET(ZB_S_FEET_DOWN_POS + 3 * f + a);
    e->md.feet_step_len[f] = GET(ZB_S_FEET_STEP_LEN + f);
    e->md.feet_f_last[f] = GET(ZB_S_FEET_F_LAST + f);
    e->md.feet_air_cur[f] = GET(ZB_S_FEET_AIR_CUR + f);
    e->md.feet_air_last[f] = GET(ZB_S_FEET_AIR_LAST + f);
    e->md.feet_contact_cur[f] = GET(ZB_S_FEET_CONTACT_CUR + f);
  }
  e->md.heading_sum = GET(ZB_S_HEADING_SUM);
  e->md.yerr_sum = GET(ZB_S_Y_ERR_SUM);
  e->md.force_sum = GET(ZB_S_FEET_FORCE_SUM);
  for (int h = 0; h < ZB_HIST; ++h) {
    e->md.feet_fz_hist[h][0] = GET(ZB_S_FEET_FZ_HIST + 2 * h);
    e->md.feet_fz_hist[h][1] = GET(ZB_S_FEET_FZ_HIST + 2 * h + 1);
    e->md.undes_fmax_hist[h] = GET(ZB_S_UNDES_FMAX_HIST + h);
  }
  e->md.ep_len = (int32_t)lrint((double)st[(size_t)ZB_S_EP_LEN * n + i]);
  for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) e->md.ep_sums[t] = GET(ZB_S_EP_SUMS + t);
#undef GET
}

int zbo_get_state(zbo_sim* s, float* dst) {
  for (int e = 0; e < s->n; ++e)
    if (s->c.task == ZB_TASK_STANDUP_V0) su_pack_env(&s->env[e], dst, s->n, e);
    else if (s->c.task == ZB_TASK_WALKING_V4) v4_pack_env(&s->env[e], dst, s->n, e);
    else if (s->c.task == ZB_TASK_MANAGER_V0) m_pack_env(&s->env[e], dst, s->n, e);
    else pack_env(&s->env[e], dst, s->n, e);
  return 0;
}
/* the persistent self-contact cache: ZB_WARM_ROWS x N floats, the kernel's layout */
int zbo_get_contact_cache(zbo_sim* s, float* dst) {
  for (int e = 0; e < s->n; ++e)
    for (int r = 0; r < ZB_WARM_ROWS; ++r) dst[(size_t)r * s->n + e] = s->env[e].wc[r];
  return 0;
}
int zbo_set_contact_cache(zbo_sim* s, const float* src) {
  for (int e = 0; e < s->n; ++e)
    for (int r = 0; r < ZB_WARM_ROWS; ++r) s->env[e].wc[r] = src[(size_t)r * s->n + e];
  return 0;
}
int zbo_set_state(zbo_sim* s, const float* src) {
  for (int e = 0; e < s->n; ++e) wc_invalidate(s->env[e].wc); /* a new state: no warm start */
  for (int e = 0; e < s->n; ++e)
    if (s->c.task == ZB_TASK_STANDUP_V0) su_unpack_env(&s->env[e], src, s->n, e);
    else if (s->c.task == ZB_TASK_WALKING_V4) v4_unpack_env(&s->env[e], src, s->n, e);
    else if (s->c.task == ZB_TASK_MANAGER_V0) m_unpack_env(&s->env[e], src, s->n, e);
    else unpack_env(&s->env[e], src, s->n, e);
  return 0;
}
int zbo_state_dim(zbo_sim* s) {
  return s->c.task == ZB_TASK_STANDUP_V0 ? ZB_SU_STATE_DIM : s->c.task == ZB_TASK_WALKING_V4 ? ZB_V4_STATE_DIM
         : s->c.task == ZB_TASK_MANAGER_V0 ? ZB_M_STATE_DIM : ZB_STATE_DIM;
}

/* standup / manager: per-link static / dynamic friction [n][12] (mu_d NULL: = mu) */
int zbo_set_link_friction(zbo_sim* s, const float* mu, const float* mu_d) {
  if (s->c.task != ZB_TASK_STANDUP_V0 && s->c.task != ZB_TASK_MANAGER_V0) return -1;
  for (int e = 0; e < s->n; ++e)
    for (int l = 0; l < NL; ++l) {
      s->env[e].md.mu[l] = mu[(size_t)e * NL + l];
      s->env[e].md.mu_d[l] = (mu_d ? mu_d : mu)[(size_t)e * NL + l];
    }
  return 0;
}

int zbo_set_link_friction_sd(zbo_sim* s, const float* mu_static, const float* mu_dynamic) {
  return zbo_set_link_friction(s, mu_static, mu_dynamic);
}

int zbo_read_curriculum(zbo_sim* s, int32_t* stage, int64_t* steps) {
  if (stage) *stage = s->stage;
  if (steps) *steps = (int64_t)s->steps;
  return 0;
}

int zbo_physics_substeps(zbo_sim* s, const float* targets, int nsub, float* net_force, float* applied_torque) {
#pragma omp parallel for schedule(static)
  for (int e = 0; e < s->n; ++e) {
    real tg[ND];
    for (int j = 0; j < ND; ++j) tg[j] = targets[(size_t)e * ND + j];
    substep_out_t so;
    memset(&so, 0, sizeof(so));
    const int dr = s->c.task == ZB_TASK_STANDUP_V0 || s->c.task == ZB_TASK_MANAGER_V0;
    const real* mu = dr ? s->env[e].md.mu : NULL;
    const real* mud = dr ? s->env[e].md.mu_d : NULL;
    clist_t wl;
    wl.n = 0;
    for (int k = 0; k < nsub; ++k) substep(&s->m, &s->c, &s->env[e].ph, tg, mu, mud, &wl, &so);
    if (net_force)
      for (int l = 0; l < NL; ++l)
        for (int a = 0; a < 3; ++a) net_force[((size_t)e * NL + l) * 3 + a] = (float)so.net_force[l][a];
    if (applied_torque)
      for (int j = 0; j < ND; ++j) applied_torque[(size_t)e * ND + j] = (float)so.applied_torque[j];
    wc_invalidate(s->env[e].wc); /* the physics moved: the cache describes another state */
  }
  return 0;
}

/* contact diagnostics of the current state (parity debugging): per env [candidates before the
 * 12-slot selection, ground candidates, self candidates (after the NSELF_MAX cap), kept, min
 * |sep - margin| over every tested ground rim point and link pair (distance to the activation
 * threshold)] */
int zbo_contact_diag(zbo_sim* s, float* out) {
  for (int e = 0; e < s->n; ++e) {
    kin_t k;
    fk(&s->m, &s->env[e].ph, &k);
    clist_t L;
    L.n = 0;
    const real margin = s->c.contact_margin;
    /* detect() without the selection, plus the threshold distance */
    real mind = 1e30;
    int ng = 0, ns = 0;
    const real Pz = s->env[e].ph.root_pos[2];
    for (int l = 0; l < NL; ++l) {
      int b = s->m.link_body[l];
      int taken = 0;
      for (int ci = 0; ci < 2; ++ci) {
        if ((s->m.circle_dup[l] >> ci) & 1) continue;
        const real* cd = s->m.circle[l][ci];
        real C[3], E1[3], E2[3];
        m3_v(k.R[b], cd, C);
        m3_v(k.R[b], cd + 3, E1);
        m3_v(k.R[b], cd + 6, E2);
        for (int a = 0; a < 3; ++a) C[a] += k.p[b][a];
        real al = -E1[2] + (real)RIM_EPS, be = -E2[2];
        real nrm = sqrtr(al * al + be * be);
        real cs = 1, sn = 0;
        if (nrm > (real)1e-12) { cs = al / nrm; sn = be / nrm; }
        const real rc[4][2] = {{cs, sn}, {-sn, cs}, {-cs, -sn}, {sn, -cs}};
        for (int r = 0; r < 4; ++r) {
          real z = C[2] + rc[r][0] * E1[2] + rc[r][1] * E2[2];
          real sep = Pz + z;
          real d = (real)fabs((double)(sep - margin));
          if (d < mind) mind = d;
          if (sep < margin && taken < NCAND_PER_LINK) { ++taken; ++ng; }
        }
      }
    }
    if (s->c.enable_self_collision) {
      for (int p = 0; p < s->m.npairs; ++p) {
        hull_t A, B;
        world_hull(&s->m, &k, s->m.pairs[p][0], &A);
        world_hull(&s->m, &k, s->m.pairs[p][1], &B);
        contact_t c;
        hull_pair(&A, &B, margin, (real)1e30, NULL, &c); /* no early exit: the separation of every pair */
        real d = (real)fabs((double)(c.sep - margin));
        if (d < mind) mind = d;
        if (c.sep < margin && ns < NSELF_MAX) ++ns;
      }
    }
    detect(&s->m, &s->c, &k, Pz, NULL, &L);
    int kself = 0; /* kept self-contact points (face manifolds count every point) */
    for (int j = 0; j < L.n; ++j) kself += L.c[j].lb >= 0;
    out[6 * e + 0] = (float)(ng + ns);
    out[6 * e + 1] = (float)ng;
    out[6 * e + 2] = (float)ns;
    out[6 * e + 3] = (float)L.n;
    out[6 * e + 4] = (float)mind;
    out[6 * e + 5] = (float)kself;
  }
  return 0;
}

/* per env, the self-contact classes of its link pairs at the current state (tests: constructed
 * manifold states, planted rare-branch bugs): out [n][10] = {pairs in contact, face-manifold pairs,
 * rim-manifold pairs (side by side, >= 2 points), overlapping-core pairs (the separating-axis
 * branch), min core separation - 2 CORE_M over the pairs, self points (cfg->self_manifold), the
 * first face pair's index (-1: none), the first rim pair's index (-1: none), ruling-on-face pairs
 * (>= 2 points), the first ruling-on-face pair's index (-1: none)} */
int zbo_pair_classes(zbo_sim* s, float* out) {
  const real margin = s->c.contact_margin;
#pragma omp parallel for schedule(dynamic, 64)
  for (int e = 0; e < s->n; ++e) {
    kin_t k;
    fk(&s->m, &s->env[e].ph, &k);
    int nh = 0, nf = 0, nr = 0, nd = 0, np_ = 0, pf = -1, pr = -1, nrf = 0, prf = -1;
    real mn = (real)1e30;
    for (int p = 0; p < s->m.npairs; ++p) {
      hull_t A, B;
      world_hull(&s->m, &k, s->m.pairs[p][0], &A);
      world_hull(&s->m, &k, s->m.pairs[p][1], &B);
      contact_t c, mf[4];
      memset(&c, 0, sizeof(c));
      const int hit = hull_pair(&A, &B, margin, margin, NULL, &c);
      if (c.sep < mn && hit) mn = c.sep;
      if (!hit) continue;
      ++nh;
      if (!(c.sep > -2 * (real)CORE_M + (real)1e-7)) ++nd;
      c.la = s->m.pairs[p][0]; c.lb = s->m.pairs[p][1];
      const int kf = s->c.self_manifold >= 1 ? self_manifold(1, &A, &B, &c, margin, mf) : 0;
      const int kr = s->c.self_manifold >= 3 && kf == 0 ? rim_face_manifold(&A, &B, &c, margin, mf) : 0;
      const int km = self_manifold(s->c.self_manifold, &A, &B, &c, margin, mf);
      if (kf > 0) { ++nf; if (pf < 0) pf = p; }
      else if (kr >= 2) { ++nrf; if (prf < 0) prf = p; }
      else if (km >= 2) { ++nr; if (pr < 0) pr = p; }
      np_ += km > 0 ? km : 1;
    }
    float* o = out + 10 * (size_t)e;
    o[0] = (float)nh; o[1] = (float)nf; o[2] = (float)nr; o[3] = (float)nd;
    o[4] = (float)(nh ? mn : 1); o[5] = (float)np_; o[6] = (float)pf; o[7] = (float)pr; o[8] = (float)nrf; o[9] = (float)prf;
  }
  return 0;
}

/* per env: the smallest self-collision separation over all link pairs (GJK on the rounded cores,
 * no early exit; -2 CORE_M = cores overlapping, beyond the exact range). Parity tests use it to
 * set aside random test states whose links interpenetrate deeper than the shape model covers. */
int zbo_self_min_sep(zbo_sim* s, float* out) {
  for (int e = 0; e < s->n; ++e) {
    kin_t k;
    fk(&s->m, &s->env[e].ph, &k);
    real mn = (real)1e30;
    for (int p = 0; p < s->m.npairs; ++p) {
      hull_t A, B;
      world_hull(&s->m, &k, s->m.pairs[p][0], &A);
      world_hull(&s->m, &k, s->m.pairs[p][1], &B);
      contact_t c;
      hull_pair(&A, &B, (real)1e30, (real)1e30, NULL, &c);
      if (c.sep < mn) mn = c.sep;
    }
    out[e] = (float)mn;
  }
  return 0;
}

/* ------------------------------------------------------------------ golden-vector entry points
 * These expose the MDP restatement on raw Isaac-Lab-shaped inputs so it can be checked against
 * vectors produced by the reference's own ZbotDirectEnvV2 code (tests/test_oracle_mdp.py). */

/* _pre_physics_step: actions [n][6] -> tanh actions, p_delta (in/out), targets */
int zbo_pre_physics(int n, const zb_task_cfg* cfg, const float* jq0, const float* actions, float* p_delta,
                    float* act_out, float* targets) {
  for (int e = 0; e < n; ++e)
    for (int j = 0; j < ND; ++j) {
      size_t i = (size_t)e * ND + j;
      real a = (real)tanh((double)actions[i]);
      real pd = (real)p_delta[i] + (real)PI_R * a * cfg->joint_speed_limit * (cfg->sim_dt * cfg->decimation);
      pd = clampr(pd, -(real)PI_R, (real)PI_R);
      p_delta[i] = (float)pd;
      act_out[i] = (float)a;
      targets[i] = (float)(pd + jq0[j]);
    }
  return 0;
}

/* cached kinematics of _get_observations from Isaac-Lab-shaped body data:
 * base/feet link pose + base COM velocity -> cache[n][24]:
 * base_pos 3, base_quat 4, fwd 3, heading_err 1, vfwd 1, feet_pos 6, feet_z 6 (-> 24) ; feet_x 6 separately */
int zbo_obs_cache(int n, const float* base_pos, const float* base_quat, const float* feet_pos, const float* feet_quat,
                  const float* base_com_vel, float* cache /*[n][30]*/) {
  for (int e = 0; e < n; ++e) {
    real bp[3], bq[4], fp[2][3], fq[2][4], bv[3];
    for (int a = 0; a < 3; ++a) { bp[a] = base_pos[e * 3 + a]; bv[a] = base_com_vel[e * 3 + a]; }
    for (int a = 0; a < 4; ++a) bq[a] = base_quat[e * 4 + a];
    for (int f = 0; f < 2; ++f) {
      for (int a = 0; a < 3; ++a) fp[f][a] = feet_pos[(e * 2 + f) * 3 + a];
      for (int a = 0; a < 4; ++a) fq[f][a] = feet_quat[(e * 2 + f) * 4 + a];
    }
    obs_cache_t o;
    make_cache(bp, bq, fp, fq, bv, &o);
    float* c = cache + (size_t)e * 30;
    for (int a = 0; a < 3; ++a) c[a] = (float)o.base_pos[a];
    for (int a = 0; a < 4; ++a) c[3 + a] = (float)o.base_quat[a];
    for (int a = 0; a < 3; ++a) c[7 + a] = (float)o.fwd[a];
    c[10] = (float)o.heading_err;
    c[11] = (float)o.vfwd;
    for (int f = 0; f < 2; ++f)
      for (int a = 0; a < 3; ++a) {
        c[12 + 3 * f + a] = (float)o.feet_pos[f][a];
        c[18 + 3 * f + a] = (float)o.feet_z[f][a];
        c[24 + 3 * f + a] = (float)o.feet_x[f][a];
      }
  }
  return 0;
}

/* _get_dones + _get_rewards on raw inputs. cache: [n][30] from zbo_obs_cache of the PREVIOUS
 * _get_observations; mdp_state: [n][13] = feet_down_pos 6, feet_step_len 2, feet_f_last 2,
 * heading_sum, yerr_sum, feet_force_sum; ep_sums [n][ZB_NUM_REWARD_TERMS] in/out. */
int zbo_mdp_eval(int n, const zb_task_cfg* cfg, const float* cache, const float* applied_torque,
                 const float* feet_vel /*[n][2][3]*/, const float* feet_fz_hist /*[n][5][2]*/,
                 const float* undes_fmax_hist /*[n][5]*/, const float* feet_air_last /*[n][2]*/,
                 const int32_t* ep_len, const float* origin_y, const float* act, const float* prev_act,
                 float* mdp_state, float* ep_sums, float* reward, float* terms, uint8_t* died, uint8_t* time_out) {
  real jq0[ND] = {0, 0, 0, 0, 0, 0};
  for (int e = 0; e < n; ++e) {
    const float* c = cache + (size_t)e * 30;
    obs_cache_t pre;
    for (int a = 0; a < 3; ++a) { pre.base_pos[a] = c[a]; pre.fwd[a] = c[7 + a]; }
    for (int a = 0; a < 4; ++a) pre.base_quat[a] = c[3 + a];
    pre.heading_err = c[10];
    pre.vfwd = c[11];
    for (int f = 0; f < 2; ++f)
      for (int a = 0; a < 3; ++a) {
        pre.feet_pos[f][a] = c[12 + 3 * f + a];
        pre.feet_z[f][a] = c[18 + 3 * f + a];
        pre.feet_x[f][a] = c[24 + 3 * f + a];
      }
    post_t ps;
    memset(&ps, 0, sizeof(ps));
    for (int j = 0; j < ND; ++j) ps.applied_torque[j] = applied_torque[(size_t)e * ND + j];
    for (int f = 0; f < 2; ++f) {
      for (int a = 0; a < 3; ++a) ps.feet_vel[f][a] = feet_vel[((size_t)e * 2 + f) * 3 + a];
      ps.feet_air_last[f] = feet_air_last[(size_t)e * 2 + f];
    }
    for (int h = 0; h < ZB_HIST; ++h) {
      ps.feet_fz_hist[h][0] = feet_fz_hist[((size_t)e * ZB_HIST + h) * 2];
      ps.feet_fz_hist[h][1] = feet_fz_hist[((size_t)e * ZB_HIST + h) * 2 + 1];
      ps.undes_fmax_hist[h] = undes_fmax_hist[(size_t)e * ZB_HIST + h];
    }
    ps.ep_len = ep_len[e];
    ps.origin_y = origin_y[e];
    mdp_t md;
    memset(&md, 0, sizeof(md));
    float* st = mdp_state + (size_t)e * 13;
    for (int f = 0; f < 2; ++f) {
      for (int a = 0; a < 3; ++a) md.feet_down_pos[f][a] = st[3 * f + a];
      md.feet_step_len[f] = st[6 + f];
      md.feet_f_last[f] = st[8 + f];
    }
    md.heading_sum = st[10];
    md.yerr_sum = st[11];
    md.force_sum = st[12];
    for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) md.ep_sums[t] = ep_sums[(size_t)e * ZB_NUM_REWARD_TERMS + t];
    real a_[ND], p_[ND], tr[ZB_NUM_REWARD_TERMS];
    for (int j = 0; j < ND; ++j) { a_[j] = act[(size_t)e * ND + j]; p_[j] = prev_act[(size_t)e * ND + j]; }
    int d = 0, to = 0;
    reward[e] = (float)mdp_eval(cfg, jq0, &pre, &ps, &md, a_, p_, tr, &d, &to);
    for (int t = 0; t < ZB_NUM_REWARD_TERMS; ++t) {
      terms[(size_t)e * ZB_NUM_REWARD_TERMS + t] = (float)tr[t];
      ep_sums[(size_t)e * ZB_NUM_REWARD_TERMS + t] = (float)md.ep_sums[t];
    }
    for (int f = 0; f < 2; ++f) {
      for (int a = 0; a < 3; ++a) st[3 * f + a] = (float)md.feet_down_pos[f][a];
      st[6 + f] = (float)md.feet_step_len[f];
      st[8 + f] = (float)md.feet_f_last[f];
    }
    st[10] = (float)md.heading_sum;
    st[11] = (float)md.yerr_sum;
    st[12] = (float)md.force_sum;
    died[e] = (uint8_t)d;
    time_out[e] = (uint8_t)to;
  }
  return 0;
}

/* world link poses for FK known-answer tests: pos [n][12][3] (env-local), quat [n][12][4] */
int zbo_link_poses(zbo_sim* s, float* pos, float* quat) {
  for (int e = 0; e < s->n; ++e) {
    kin_t k;
    fk(&s->m, &s->env[e].ph, &k);
    for (int l = 0; l < NL; ++l) {
      real p[3], q[4];
      link_pose(&s->m, &k, l, p, q);
      for (int a = 0; a < 3; ++a) pos[((size_t)e * NL + l) * 3 + a] = (float)(p[a] + s->env[e].ph.root_pos[a]);
      for (int a = 0; a < 4; ++a) quat[((size_t)e * NL + l) * 4 + a] = (float)q[a];
    }
  }
  return 0;
}

/* link COM linear velocities [n][12][3] (body_com_lin_vel_w) */
int zbo_link_com_vel(zbo_sim* s, float* vel) {
  for (int e = 0; e < s->n; ++e) {
    kin_t k;
    fk(&s->m, &s->env[e].ph, &k);
    real V[NB][6];
    body_vel(&k, &s->env[e].ph, V);
    for (int l = 0; l < NL; ++l) {
      int b = s->m.link_body[l];
      real c[3], v[3];
      m3_v(k.R[b], s->m.link_com[l], c);
      for (int a = 0; a < 3; ++a) c[a] += k.p[b][a];
      point_vel(V[b], c, v);
      for (int a = 0; a < 3; ++a) vel[((size_t)e * NL + l) * 3 + a] = (float)v[a];
    }
  }
  return 0;
}

/* total mechanical energy and momentum (invariant tests): out[n][7] = E, p(3), L_about_origin(3) */
int zbo_energy_momentum(zbo_sim* s, float* out) {
  for (int e = 0; e < s->n; ++e) {
    const phys_t* ph = &s->env[e].ph;
    kin_t k;
    fk(&s->m, ph, &k);
    real V[NB][6];
    body_vel(&k, ph, V);
    real E = 0, P[3] = {0, 0, 0}, Lm[3] = {0, 0, 0};
    for (int b = 0; b < NB; ++b) {
      sinertia I;
      body_sinertia(&s->m, &k, b, &I);
      real f[6];
      si_mul(&I, V[b], f);
      E += (real)0.5 * (f[0] * V[b][0] + f[1] * V[b][1] + f[2] * V[b][2] + f[3] * V[b][3] + f[4] * V[b][4] + f[5] * V[b][5]);
      real cz = I.h[2] / I.m + ph->root_pos[2];
      E += I.m * s->c.gravity * cz;
      for (int a = 0; a < 3; ++a) { P[a] += f[3 + a]; Lm[a] += f[a]; }
    }
    /* angular momentum about the world origin: L_O = L_P + P_root x p */
    real rp[3];
    v3_cross(ph->root_pos, P, rp);
    out[(size_t)e * 7] = (float)E;
    for (int a = 0; a < 3; ++a) { out[(size_t)e * 7 + 1 + a] = (float)P[a]; out[(size_t)e * 7 + 4 + a] = (float)(Lm[a] + rp[a]); }
  }
  return 0;
}

/* Stand-up MDP on raw Isaac-Lab-shaped inputs (golden vectors from the reference's own
 * Zbot6SUpEnv code, tests/test_oracle_standup.py): link_state [n][12][13] = body_link_state_w
 * (pos 3, quat 4, lin vel 3, ang vel 3), p_delta [n][6] after _pre_physics_step, ep_len [n]
 * after the += 1, center_z_last [n] in/out, ep_sums [n][4] in/out. */
int zbo_su_mdp_eval(int n, const zb_task_cfg* cfg, int stage, const float* link_state, const float* p_delta,
                    const int32_t* ep_len, float* center_z_last, float* ep_sums, float* reward, float* terms,
                    uint8_t* died, uint8_t* time_out) {
  for (int e = 0; e < n; ++e) {
    const float* ls = link_state + (size_t)e * NL * 13;
    su_links_t L;
    L.z4 = ls[4 * 13 + 2]; L.z6 = ls[6 * 13 + 2]; L.z8 = ls[8 * 13 + 2];
    L.vz5 = ls[5 * 13 + 9]; L.vz6 = ls[6 * 13 + 9];
    for (int a = 0; a < 4; ++a) {
      L.feet_quat[0][a] = ls[0 * 13 + 3 + a];
      L.feet_quat[1][a] = ls[11 * 13 + 3 + a];
      L.base_quat[a] = ls[6 * 13 + 3 + a];
    }
    real pd[ND], sums[ZB_SU_NUM_REWARD_TERMS], tr[ZB_SU_NUM_REWARD_TERMS];
    for (int j = 0; j < ND; ++j) pd[j] = p_delta[(size_t)e * ND + j];
    for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) sums[t] = ep_sums[(size_t)e * ZB_SU_NUM_REWARD_TERMS + t];
    real czl = center_z_last[e];
    int d = 0, to = 0;
    reward[e] = (float)su_mdp_eval(cfg, stage, &L, pd, ep_len[e], &czl, sums, tr, &d, &to);
    center_z_last[e] = (float)czl;
    for (int t = 0; t < ZB_SU_NUM_REWARD_TERMS; ++t) {
      terms[(size_t)e * ZB_SU_NUM_REWARD_TERMS + t] = (float)tr[t];
      ep_sums[(size_t)e * ZB_SU_NUM_REWARD_TERMS + t] = (float)sums[t];
    }
    died[e] = (uint8_t)d;
    time_out[e] = (uint8_t)to;
  }
  return 0;
}

/* reset_root_state_uniform draws (root pos [n][3], quat [n][4]) at RNG position ctr */
int zbo_su_reset_pose(const zb_model* model, const zb_task_cfg* cfg, uint64_t seed, uint64_t ctr, int n, float* pos,
                      float* quat) {
  mdl_t m;
  load_mdl(model, &m);
  for (int e = 0; e < n; ++e) {
    phys_t p;
    su_reset_pose(&m, cfg, seed, ctr, e, &p);
    for (int a = 0; a < 3; ++a) pos[(size_t)e * 3 + a] = (float)p.root_pos[a];
    for (int a = 0; a < 4; ++a) quat[(size_t)e * 4 + a] = (float)p.root_quat[a];
  }
  return 0;
}

/* root pose from reset_root_state_uniform samples [n][4] = (x, y, roll, yaw) */
int zbo_su_pose_from_samples(const zb_model* model, int n, const float* samples, int body_frame, float* pos,
                             float* quat) {
  mdl_t m;
  load_mdl(model, &m);
  for (int e = 0; e < n; ++e) {
    phys_t p;
    real r[4];
    for (int k = 0; k < 4; ++k) r[k] = samples[(size_t)e * 4 + k];
    pose_from_samples(&m, r, body_frame, &p);
    for (int a = 0; a < 3; ++a) pos[(size_t)e * 3 + a] = (float)p.root_pos[a];
    for (int a = 0; a < 4; ++a) quat[(size_t)e * 4 + a] = (float)p.root_quat[a];
  }
  return 0;
}

/* ------------------------------------------------------------------ v4 golden-vector entry points */

/* v4 _get_dones + _get_rewards on Isaac-Lab-shaped data (tests/test_oracle_v4.py):
 * link_pos [n][12][3], link_quat [n][12][4], link_lin_vel [n][12][3] (body_link_lin_vel_w),
 * com_lin_vel [n][12][3] (body_com_lin_vel_w), joint_vel / joint_acc / applied_torque [n][6],
 * net_forces_hist [n][3][12][3], sensor times [n][12] x 4 (current air, current contact, last air,
 * last contact), ep_len [n] (after += 1), actions / prev actions [n][6]; in/out commands [n][2],
 * target_yaw [n], feet_down_pos [n][2][3], feet_step_len [n][2], feet_f_last [n][2], ep_sums [n][15]. */
int zbo_v4_mdp_eval(int n, const zb_task_cfg* cfg, int stage, const zb_model* model, const float* link_pos,
                    const float* link_quat, const float* link_lin_vel, const float* com_lin_vel, const float* joint_vel,
                    const float* joint_acc, const float* applied_torque, const float* net_forces_hist,
                    const float* air_cur, const float* con_cur, const float* air_last, const float* con_last,
                    const int32_t* ep_len, const float* act, const float* prev_act, const float* commands,
                    const float* target_yaw, float* feet_down_pos, float* feet_step_len, float* feet_f_last,
                    float* ep_sums, float* reward, float* terms, uint8_t* died, uint8_t* time_out, float* cur_yaw,
                    float* heading_err) {
  mdl_t m;
  load_mdl(model, &m);
  for (int e = 0; e < n; ++e) {
    v4_post_t P;
    const int B = m.base_link;
    for (int a = 0; a < 3; ++a) {
      P.base_pos[a] = link_pos[((size_t)e * NL + B) * 3 + a];
      P.base_lin_vel[a] = link_lin_vel[((size_t)e * NL + B) * 3 + a];
    }
    for (int a = 0; a < 4; ++a) P.base_quat[a] = link_quat[((size_t)e * NL + B) * 4 + a];
    for (int f = 0; f < 2; ++f) {
      const int l = m.foot_links[f];
      for (int a = 0; a < 3; ++a) {
        P.feet_pos[f][a] = link_pos[((size_t)e * NL + l) * 3 + a];
        P.feet_com_vel[f][a] = com_lin_vel[((size_t)e * NL + l) * 3 + a];
      }
      for (int a = 0; a < 4; ++a) P.feet_quat[f][a] = link_quat[((size_t)e * NL + l) * 4 + a];
      P.air_cur[f] = air_cur[(size_t)e * NL + l]; P.con_cur[f] = con_cur[(size_t)e * NL + l];
      P.air_last[f] = air_last[(size_t)e * NL + l]; P.con_last[f] = con_last[(size_t)e * NL + l];
    }
    for (int j = 0; j < ND; ++j) {
      P.jqd[j] = joint_vel[(size_t)e * ND + j];
      P.joint_acc[j] = joint_acc[(size_t)e * ND + j];
      P.applied_torque[j] = applied_torque[(size_t)e * ND + j];
    }
    for (int h = 0; h < ZB_V4_HIST; ++h) {
      const float* F = net_forces_hist + ((size_t)e * ZB_V4_HIST + h) * NL * 3;
      P.fz_hist[h][0] = F[m.foot_links[0] * 3 + 2];
      P.fz_hist[h][1] = F[m.foot_links[1] * 3 + 2];
      real fm = 0;
      for (int k = 0; k < 10; ++k) {
        const float* f3 = F + m.undesired[k] * 3;
        const real nrm = sqrtr((real)f3[0] * f3[0] + (real)f3[1] * f3[1] + (real)f3[2] * f3[2]);
        if (nrm > fm) fm = nrm;
      }
      P.undes_fmax_hist[h] = fm;
    }
    P.ep_len = ep_len[e];
    mdp_t md;
    memset(&md, 0, sizeof(md));
    md.commands[0] = commands[(size_t)e * 2]; md.commands[1] = commands[(size_t)e * 2 + 1];
    md.target_yaw = target_yaw[e];
    for (int f = 0; f < 2; ++f) {
      for (int a = 0; a < 3; ++a) md.feet_down_pos[f][a] = feet_down_pos[((size_t)e * 2 + f) * 3 + a];
      md.feet_step_len[f] = feet_step_len[(size_t)e * 2 + f];
      md.feet_f_last[f] = feet_f_last[(size_t)e * 2 + f];
    }
    for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) md.ep_sums[t] = ep_sums[(size_t)e * ZB_V4_NUM_REWARD_TERMS + t];
    real a_[ND], p_[ND], tr[ZB_V4_NUM_REWARD_TERMS];
    for (int j = 0; j < ND; ++j) { a_[j] = act[(size_t)e * ND + j]; p_[j] = prev_act[(size_t)e * ND + j]; }
    int d = 0, to = 0;
    v4_aux_t aux;
    reward[e] = (float)v4_mdp_eval(cfg, stage, &P, &md, a_, p_, tr, &d, &to, &aux);
    for (int t = 0; t < ZB_V4_NUM_REWARD_TERMS; ++t) {
      terms[(size_t)e * ZB_V4_NUM_REWARD_TERMS + t] = (float)tr[t];
      ep_sums[(size_t)e * ZB_V4_NUM_REWARD_TERMS + t] = (float)md.ep_sums[t];
    }
    for (int f = 0; f < 2; ++f) {
      for (int a = 0; a < 3; ++a) feet_down_pos[((size_t)e * 2 + f) * 3 + a] = (float)md.feet_down_pos[f][a];
      feet_step_len[(size_t)e * 2 + f] = (float)md.feet_step_len[f];
      feet_f_last[(size_t)e * 2 + f] = (float)md.feet_f_last[f];
    }
    died[e] = (uint8_t)d;
    time_out[e] = (uint8_t)to;
    cur_yaw[e] = (float)aux.cur_yaw;
    heading_err[e] = (float)aux.heading_err;
  }
  return 0;
}

/* resample_commands on given draws: params = {prob_pos, vel lo, vel hi, yaw lo, yaw hi, offset} */
int zbo_v4_commands_from_draws(int n, const float* params, const float* u_sign, const float* u_vel, const float* u_yaw,
                               const float* cur_yaw, float* cmd, float* target) {
  const float vr[2] = {params[1], params[2]}, yr[2] = {params[3], params[4]};
  for (int e = 0; e < n; ++e) {
    real c[2], t;
    v4_commands(1, params[0], vr, yr, params[5], u_sign[e], u_vel[e], u_yaw[e], cur_yaw[e], c, &t);
    cmd[(size_t)e * 2] = (float)c[0];
    cmd[(size_t)e * 2 + 1] = (float)c[1];
    target[e] = (float)t;
  }
  return 0;
}

/* the reset-event curricula on a given counter state: io = {stage, prob_pos, vel lo, vel hi, yaw lo,
 * yaw hi} in / out; the range buffers hold ring_n copies of (ring_vel, ring_yaw) */
int zbo_curriculum_probe(const zb_task_cfg* cfg, int64_t steps, int run_my, int run_range, int ring_n, float ring_vel,
                         float ring_yaw, float* io) {
  zbo_sim s;
  memset(&s, 0, sizeof(s));
  s.c = *cfg;
  s.steps = (uint64_t)steps;
  s.stage = (int)io[0];
  s.prob_pos = io[1];
  s.vel[0] = io[2]; s.vel[1] = io[3]; s.yaw[0] = io[4]; s.yaw[1] = io[5];
  s.ring_n = ring_n;
  for (int k = 0; k < ring_n; ++k) { s.ring_vel[k] = ring_vel; s.ring_yaw[k] = ring_yaw; }
  curriculum_events(&s, run_my, run_range);
  io[0] = (float)s.stage; io[1] = s.prob_pos;
  io[2] = s.vel[0]; io[3] = s.vel[1]; io[4] = s.yaw[0]; io[5] = s.yaw[1];
  return 0;
}

/* manager flat MDP (terminations + rewards) on Isaac-Lab-shaped inputs, per env:
 * base_pos[3], base_quat[4], base_lin_vel[3] (root_link_lin_vel_w), base_ang_vel[3]
 * (root_link_ang_vel_w), feet_pos[2][3], feet_quat[2][4], feet_vel[2][3] (body_lin_vel_w),
 * net_forces_w_history of the feet [3][2][3], last_air_time[2], applied_torque[6], joint_acc[6],
 * ep_len, actions / prev actions [6]; state in/out: commands[3], feet_down_pos[2][3],
 * feet_step_len[2], feet_f_last[2], ep_sums[11]; out: reward, terms[11], low, close, time_out */
int zbo_m_mdp_eval(int n, const zb_task_cfg* cfg, const float* base_pos, const float* base_quat, const float* base_lin_vel,
                   const float* base_ang_vel, const float* feet_pos, const float* feet_quat, const float* feet_vel,
                   const float* hist, const float* air_last, const float* applied_torque, const float* joint_acc,
                   const int32_t* ep_len, const float* act, const float* prev, const float* commands,
                   float* feet_down_pos, float* feet_step_len, float* feet_f_last, float* ep_sums, float* reward,
                   float* terms, uint8_t* low, uint8_t* close, uint8_t* tout) {
  for (int e = 0; e < n; ++e) {
    m_post_t P;
    mdp_t md;
    memset(&md, 0, sizeof(md));
    for (int a = 0; a < 3; ++a) {
      P.base_pos[a] = base_pos[3 * e + a];
      P.base_lin_vel[a] = base_lin_vel[3 * e + a];
      P.base_ang_vel[a] = base_ang_vel[3 * e + a];
      md.commands[a] = commands[3 * e + a];
    }
    for (int a = 0; a < 4; ++a) P.base_quat[a] = base_quat[4 * e + a];
    for (int f = 0; f < 2; ++f) {
      for (int a = 0; a < 3; ++a) {
        P.feet_pos[f][a] = feet_pos[6 * e + 3 * f + a];
        P.feet_vel[f][a] = feet_vel[6 * e + 3 * f + a];
        md.feet_down_pos[f][a] = feet_down_pos[6 * e + 3 * f + a];
      }
      for (int a = 0; a < 4; ++a) P.feet_quat[f][a] = feet_quat[8 * e + 4 * f + a];
      for (int h = 0; h < 3; ++h) {
        const float* F = hist + (size_t)e * 18 + h * 6 + f * 3;
        P.fz_hist[h][f] = F[2];
        P.fn_hist[h][f] = sqrtr((real)F[0] * F[0] + (real)F[1] * F[1] + (real)F[2] * F[2]);
      }
      P.air_last[f] = air_last[2 * e + f];
      md.feet_step_len[f] = feet_step_len[2 * e + f];
      md.feet_f_last[f] = feet_f_last[2 * e + f];
    }
    real a6[ND], p6[ND];
    for (int j = 0; j < ND; ++j) {
      P.applied_torque[j] = applied_torque[6 * e + j];
      P.joint_acc[j] = joint_acc[6 * e + j];
      a6[j] = act[6 * e + j];
      p6[j] = prev[6 * e + j];
    }
    P.ep_len = ep_len[e];
    for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) md.ep_sums[t] = ep_sums[ZB_M_NUM_REWARD_TERMS * e + t];
    real tm[ZB_M_NUM_REWARD_TERMS];
    int lo = 0, cl = 0, to = 0;
    reward[e] = (float)m_mdp_eval(cfg, &P, &md, a6, p6, tm, &lo, &cl, &to);
    for (int t = 0; t < ZB_M_NUM_REWARD_TERMS; ++t) {
      terms[ZB_M_NUM_REWARD_TERMS * e + t] = (float)tm[t];
      ep_sums[ZB_M_NUM_REWARD_TERMS * e + t] = (float)md.ep_sums[t];
    }
    for (int f = 0; f < 2; ++f) {
      for (int a = 0; a < 3; ++a) feet_down_pos[6 * e + 3 * f + a] = (float)md.feet_down_pos[f][a];
      feet_step_len[2 * e + f] = (float)md.feet_step_len[f];
      feet_f_last[2 * e + f] = (float)md.feet_f_last[f];
    }
    low[e] = (uint8_t)lo;
    close[e] = (uint8_t)cl;
    tout[e] = (uint8_t)to;
  }
  return 0;
}

/* lin_vel_cmd_levels on io = [x lo, x hi, y lo, y hi] (in/out); returns 1 if it fired */
int zbo_m_curriculum_probe(const zb_task_cfg* cfg, int64_t steps, float reward, float* io) {
  float vel[2] = {io[0], io[1]}, yaw[2] = {io[2], io[3]};
  const int r = m_lin_vel_cmd_levels(cfg, (uint64_t)steps, reward, vel, yaw);
  io[0] = vel[0]; io[1] = vel[1]; io[2] = yaw[0]; io[3] = yaw[1];
  return r;
}

/* RelativeJointPositionAction: raw actions [n][6] (Isaac Lab joint order) -> processed actions
 * (scale, clip) in the Isaac Lab order and the per-substep targets q + delta of the chain joints */
int zbo_m_process_actions(int n, const zb_task_cfg* cfg, const zb_model* model, const float* actions, const float* jq,
                          float* processed, float* targets) {
  mdl_t m;
  load_mdl(model, &m);
  for (int e = 0; e < n; ++e) {
    for (int a = 0; a < ND; ++a)
      processed[6 * e + a] = (float)clampr((real)actions[6 * e + a] * (real)cfg->action_scale, -(real)cfg->action_clip,
                                           (real)cfg->action_clip);
    for (int j = 0; j < ND; ++j)
      targets[6 * e + j] = (float)((real)jq[6 * e + j] + m.api_sign[j] * (real)processed[6 * e + m.api_index[j]]);
  }
  return 0;
}
