/*
 * zbot.h — C ABI of the MI355X-native batched ZBOT-6 simulator: zbot-6b-walking-v2 (the hot path)
 * and zbot-6b-standup-v0 (the snake -> biped stand-up task on the same robot and physics).
 *
 * One handle owns N environments' persistent state in HBM (SoA, [field][env], fp32) and steps
 * them with one fused HIP kernel per policy step (4 physics substeps + contact sensor + MDP +
 * in-kernel auto-reset). The CPU oracle (oracle/zbot_oracle.c) exports the same entry points with
 * the prefix `zbo_` and host pointers; it is test infrastructure only.
 *
 * Reference interfaces replaced (paths relative to the reference repo root):
 *   zb_create   <- gym.make("zbot-6b-walking-v2") -> ZbotDirectEnvV2.__init__
 *                  (source/zbot/zbot/tasks/zbot6b_direct/__init__.py:41-49;
 *                   .../zbot_direct_6dof_bipedal_env_v2.py:211-257, _setup_scene 259-274)
 *   zb_reset    <- DirectRLEnv.reset() -> ZbotDirectEnvV2._reset_idx (v2.py:413-459)
 *   zb_step     <- DirectRLEnv.step(a): _pre_physics_step (v2.py:276-287), 4 x {_apply_action
 *                  (v2.py:309-310), PhysX sim.step, scene.update}, _get_dones (v2.py:384-411),
 *                  _get_rewards (v2.py:371-382), _reset_idx (v2.py:413-459),
 *                  _get_observations (v2.py:312-369)
 *   zb_observe  <- ZbotDirectEnvV2._get_observations (v2.py:312-369), used by reset()
 *   zb_read_log / zb_set_log_buffers <- extras["log"] written in _reset_idx (v2.py:441-459)
 *   zb_get_state / zb_set_state / zb_physics_substeps: parity + debugging (no reference analogue;
 *                  they stand in for Articulation.data reads / write_*_to_sim)
 *
 * Stand-up task (task = ZB_TASK_STANDUP_V0; source/zbot/zbot/tasks/zbot6b_direct/
 * zbot_direct_6_standup_env_v0.py = "standup.py", robot ZBOT_6S_CFG_2 zbot_cfg.py:721-763):
 *   zb_create   <- gym.make("zbot-6b-standup-v0") -> Zbot6SUpEnv.__init__ (standup.py:453-535)
 *   zb_step     <- _pre_physics_step (538-551), 4 x physics, _get_dones (634-643) with
 *                  _compute_intermediate_values (571-591), _get_rewards (620-632, terms 705-856),
 *                  _reset_idx (645-703) incl. the reset events reset_root_state_uniform (33-97)
 *                  and my_curriculum (99-111), _get_observations (593-618)
 *   zb_set_link_friction <- EventCfg.physics_material = randomize_rigid_body_material
 *                  (startup event, standup.py:124-136): the sampled per-shape friction
 *   zb_read_curriculum <- Zbot6SUpEnv.curriculum_stage / common_step_counter
 *
 * Conventions: quaternions (w, x, y, z); world Z-up; gravity (0, 0, -9.81); every env in its
 * own env-local frame (origin 0; the plane is infinite and envs are collision-filtered in the
 * reference, v2.py:271, so physics is translation invariant).
 * All device entry points are stream-ordered and never synchronise the host. Return 0 on
 * success, a negative code on error (message via zb_last_error()). Not thread-safe per handle.
 */
#ifndef ZBOT_H_
#define ZBOT_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZB_NUM_LINKS 12       /* foot_0 b1 a2 b2 a3 b3 base b4 a5 b5 a6 foot_1 */
#define ZB_NUM_BODIES 7       /* rigid composites after merging the 5 fixed joints */
#define ZB_NUM_DOF 6          /* revolute joint1..joint6 */
#define ZB_ACT_DIM 6
#define ZB_OBS_DIM 23
#define ZB_NUM_REWARD_TERMS 15  /* step4's 13 (v2.py:190-206) + step0's feet_force_diff / feet_force_sum (v2.py:78-91) */
#define ZB_HIST 5             /* contact sensor history_length (v2.py:32) */
#define ZB_MAX_SELF_PAIRS 64
#ifndef ZB_MAX_CONTACTS
#define ZB_MAX_CONTACTS 12    /* contact slots per env per substep (deepest kept); -D for the cap A/B build (<= 16) */
#endif

#define ZB_WARM_SLOTS 4       /* persistent self-contact cache: kept self contacts carried to the next step */
#define ZB_WARM_ROWS (4 * ZB_WARM_SLOTS) /* {n.x, n.y, n.z, code} per slot (code -1: none), rows x N */

#define ZB_TASK_WALKING_V2 0  /* zbot-6b-walking-v2 (v2.py) */
#define ZB_TASK_STANDUP_V0 1  /* zbot-6b-standup-v0 (standup.py) */
#define ZB_TASK_WALKING_V4 2  /* zbot-6b-walking-v4 (v4.py): v2 + commands, events, curricula */
#define ZB_TASK_MANAGER_V0 3  /* zbot-6b-walking-m-v0: the manager-based flat env (zbotlab_env_cfg.py) */
#define ZB_M_OBS_DIM 25       /* base quat 4, velocity command 3, joint pos 6, joint vel 6, last action 6 */
#define ZB_M_NUM_REWARD_TERMS 11
#define ZB_SU_OBS_DIM 22      /* standup.py:199 */
#define ZB_SU_NUM_REWARD_TERMS 4
#define ZB_V4_OBS_DIM 24      /* v4.py:453 */
#define ZB_V4_NUM_REWARD_TERMS 15
#define ZB_V4_HIST 3          /* v4 contact sensor history_length (v4.py:522) */
#define ZB_MAX_REWARD_TERMS 16
#define ZB_MAX_STAGES 4       /* curriculum stages */
#define ZB_V4_RING 24         /* range_curriculum reward buffers: deque(maxlen=24) (v4.py:700-701) */
/* Episode log buffer (zb_read_log): [0..15] Episode_Reward/<term> means in term order,
 * [16] Curriculum/curriculum_stage, [17..18] Curriculum/vel_lower_bound, vel_upper_bound,
 * [19] Curriculum/yaw_bound (v4 only; v4.py:952-957) */
#define ZB_LOG_LEN 20
/* Termination counts (zb_read_log counts[ZB_LOG_COUNTS]): walking v2 {body_contact, time_out},
 * standup / v4 {died, time_out}, manager {base_height, time_out, feet_close}; the manager's log
 * floats [16..18] are Curriculum/lin_vel_cmd_levels, Metrics/base_velocity/error_vel_xy, error_vel_yaw */
#define ZB_LOG_COUNTS 4

/* Persistent per-env state, SoA [ZB_STATE_DIM][num_envs] float32. */
enum zb_state_field {
  ZB_S_ROOT_POS = 0,        /* 3  root link (foot_0) origin, env-local */
  ZB_S_ROOT_QUAT = 3,       /* 4  wxyz */
  ZB_S_ROOT_LINVEL = 7,     /* 3  world velocity of the root link origin */
  ZB_S_ROOT_ANGVEL = 10,    /* 3  world */
  ZB_S_JOINT_POS = 13,      /* 6 */
  ZB_S_JOINT_VEL = 19,      /* 6 */
  ZB_S_P_DELTA = 25,        /* 6  v2.py:245,280-286 */
  ZB_S_ACTIONS = 31,        /* 6  tanh(actions) of the last step (= _previous_actions next step) */
  ZB_S_FEET_DOWN_POS = 37,  /* 6  [foot][xyz] v2.py:235 */
  ZB_S_FEET_STEP_LEN = 43,  /* 2  v2.py:236 */
  ZB_S_FEET_F_LAST = 45,    /* 2  v2.py:231 */
  ZB_S_HEADING_SUM = 47,    /* 1  v2.py:239 */
  ZB_S_Y_ERR_SUM = 48,      /* 1  v2.py:240 */
  ZB_S_FEET_FZ_HIST = 49,   /* 10 [slot][foot], slot 0 newest: net_forces_w_history[..., feet, 2] */
  ZB_S_UNDES_FMAX_HIST = 59,/* 5  [slot]: max over the 10 undesired bodies of |net force| */
  ZB_S_FEET_AIR_CUR = 64,   /* 2  ContactSensor current_air_time[feet] */
  ZB_S_FEET_AIR_LAST = 66,  /* 2  last_air_time[feet] */
  ZB_S_FEET_CONTACT_CUR = 68,/*2  current_contact_time[feet] */
  ZB_S_EP_LEN = 70,         /* 1  episode_length_buf (integer-valued float) */
  ZB_S_EP_SUMS = 71,        /* 15 _episode_sums in reward-term order */
  ZB_S_FEET_FORCE_SUM = 86, /* 1  v2.py:238 (step0's feet_force_sum integrator, zeroed on reset :437) */
  ZB_STATE_DIM = 87
};

/* Stand-up task state, SoA [ZB_SU_STATE_DIM][num_envs] float32. Rows 0..24 (root, joints) are
 * laid out as in zb_state_field. */
enum zb_standup_state_field {
  ZB_SU_P_DELTA = 25,       /* 6  standup.py:484,540-548 */
  ZB_SU_ACTIONS = 31,       /* 6  tanh(actions) of the last step */
  ZB_SU_CENTER_Z_LAST = 37, /* 1  standup.py:511,639-641 */
  ZB_SU_EP_LEN = 38,        /* 1  episode_length_buf (integer-valued float) */
  ZB_SU_EP_SUMS = 39,       /* 4  _episode_sums in reward-term order */
  ZB_SU_LINK_MU = 43,       /* 12 per-link static friction coefficient (read-only for zb_step) */
  ZB_SU_LINK_MU_D = 55,     /* 12 per-link dynamic friction coefficient (read-only for zb_step) */
  ZB_SU_STATE_DIM = 67
};

/* v4 state, SoA [ZB_V4_STATE_DIM][num_envs] float32; rows 0..24 as in zb_state_field. */
enum zb_v4_state_field {
  ZB_V4_P_DELTA = 25,         /* 6 */
  ZB_V4_ACTIONS = 31,         /* 6 */
  ZB_V4_COMMANDS = 37,        /* 2  commands: target forward velocity, relative yaw (v4.py:697) */
  ZB_V4_TARGET_YAW = 39,      /* 1  target_heading_yaw (world, v4.py:699) */
  ZB_V4_INTERVAL_LEFT = 40,   /* 1  interval_command_resample time left (s) */
  ZB_V4_FEET_DOWN_POS = 41,   /* 6 */
  ZB_V4_FEET_STEP_LEN = 47,   /* 2 */
  ZB_V4_FEET_F_LAST = 49,     /* 2 */
  ZB_V4_FEET_FZ_HIST = 51,    /* 6  [slot][foot], slot 0 newest */
  ZB_V4_UNDES_FMAX_HIST = 57, /* 3 */
  ZB_V4_FEET_AIR_CUR = 60,    /* 2 */
  ZB_V4_FEET_CONTACT_CUR = 62,/* 2 */
  ZB_V4_FEET_AIR_LAST = 64,   /* 2 */
  ZB_V4_FEET_CONTACT_LAST = 66,/*2 */
  ZB_V4_EP_LEN = 68,          /* 1 */
  ZB_V4_EP_SUMS = 69,         /* 15 */
  ZB_V4_CURRENT_YAW = 84,     /* 1  current_yaw: post-step heading, or the reset event's yaw sample */
  ZB_V4_STATE_DIM = 85
};

/* Manager-based flat env state (zbot-6b-walking-m-v0), SoA [ZB_M_STATE_DIM][num_envs]; rows 0..24
 * are the internal chain's physics state as in zb_state_field (the Isaac Lab root is the base link,
 * see zb_model.api_root_*). */
enum zb_manager_state_field {
  ZB_M_ACTIONS = 25,          /* 6  raw actions of the last step, Isaac Lab joint order (last_action) */
  ZB_M_COMMANDS = 31,         /* 3  base_velocity command (lin x, lin y, ang z) */
  ZB_M_CMD_TIME_LEFT = 34,    /* 1  command resampling timer (s) */
  ZB_M_CMD_STANDING = 35,     /* 1  is_standing_env (0 / 1) */
  ZB_M_FEET_DOWN_POS = 36,    /* 6  env.feet_down_pos_last (rewards.py:29-35) */
  ZB_M_FEET_STEP_LEN = 42,    /* 2 */
  ZB_M_FEET_F_LAST = 44,      /* 2 */
  ZB_M_FEET_FZ_HIST = 46,     /* 6  [slot][foot] net_forces_w_history[..., feet, 2], slot 0 newest; the
                                 sensor (history 3) updates every physics step: substeps 4, 3, 2 */
  ZB_M_FEET_FN_HIST = 52,     /* 6  [slot][foot] |net force| of the feet */
  ZB_M_FEET_AIR_CUR = 58,     /* 2 */
  ZB_M_FEET_AIR_LAST = 60,    /* 2 */
  ZB_M_METRICS = 62,          /* 2  command metrics error_vel_xy, error_vel_yaw */
  ZB_M_EP_LEN = 64,           /* 1 */
  ZB_M_EP_SUMS = 65,          /* 11 reward manager episode sums */
  ZB_M_LINK_MU = 76,          /* 12 per-link static friction (physics_material startup event) */
  ZB_M_LINK_MU_D = 88,        /* 12 per-link dynamic friction */
  ZB_M_STATE_DIM = 100
};

/* Manager reward term order = RewardsCfg field order of Zbot6BFlatEnvCfg (zbotlab_env_cfg.py,
 * flat_env_cfg.py) with the terms the flat cfg sets to None removed
 * (zbotlab_env_cfg.py:261-377, flat_env_cfg.py:169-182). */
enum zb_manager_reward_term {
  ZB_M_R_TRACK_LIN_VEL_XY = 0, ZB_M_R_TRACK_ANG_VEL_Z, ZB_M_R_TERMINATION, ZB_M_R_DOF_TORQUES, ZB_M_R_DOF_ACC,
  ZB_M_R_ACTION_RATE, ZB_M_R_FOOT_STEP_LENGTH, ZB_M_R_FOOT_DOWNWARD, ZB_M_R_FOOT_FORWARD, ZB_M_R_FEET_SLIDE,
  ZB_M_R_AIR_TIME_BALANCE
};

/* v4 reward term order = dict order of Zbot6SEnvV4Cfg.reward_cfg (v4.py:620-641). */
enum zb_v4_reward_term {
  ZB_V4_R_TRACK_LIN_VEL_X = 0, ZB_V4_R_TRACK_HEADING_YAW, ZB_V4_R_LIN_VEL_Y, ZB_V4_R_ACTION_RATE, ZB_V4_R_TORQUES,
  ZB_V4_R_JOINT_VEL, ZB_V4_R_JOINT_ACC, ZB_V4_R_FEET_DOWNWARD, ZB_V4_R_FEET_FORWARD, ZB_V4_R_STEP_LENGTH,
  ZB_V4_R_FEET_AIR_TIME_BIPED, ZB_V4_R_AIRTIME_VARIANCE, ZB_V4_R_FEET_SLIDE, ZB_V4_R_FEET_HARMONY, ZB_V4_R_FEET_CLOSE
};

/* Stand-up reward term order = dict order of Zbot6SUpEnvCfg.reward_cfg (standup.py:418-427). */
enum zb_standup_reward_term {
  ZB_SU_R_UPWARD_2 = 0, ZB_SU_R_SHAPE_SYMMETRY, ZB_SU_R_FEET_DOWNWARD, ZB_SU_R_FEET_DOWNWARD_4
};

/* Reward term order = dict order of ZbotDirectEnvCfgV2.reward_cfg (v2.py:190-206), then step0's two
 * feet-force terms (v2.py:78-91, 563-571; feet_force_diff before feet_force_sum, as in that dict). */
enum zb_reward_term {
  ZB_R_BASE_VEL_FORWARD = 0, ZB_R_FEET_DOWNWARD, ZB_R_FEET_FORWARD, ZB_R_BASE_HEADING_X,
  ZB_R_BASE_HEADING_X_SUM, ZB_R_STEP_LENGTH, ZB_R_AIRTIME_BALANCE, ZB_R_ACTION_RATE,
  ZB_R_TORQUES, ZB_R_FEET_SLIDE, ZB_R_BASE_POS_Y_ERR, ZB_R_BASE_POS_Y_ERR_SUM, ZB_R_AIRTIME_SUM,
  ZB_R_FEET_FORCE_DIFF, ZB_R_FEET_FORCE_SUM
};

/* Robot model: ZBOT_6S_CFG (zbot_cfg.py:621-669) + zbot_6s_new.usd, fixed joints merged.
 * Filled by zbot_lab_amd/model.py from zbot_lab_amd/assets/zbot6s_model.json. */
typedef struct zb_model {
  /* composite rigid bodies; body b>0 hangs off body b-1 through revolute joint b-1 */
  float body_mass[ZB_NUM_BODIES];
  float body_com[ZB_NUM_BODIES][3];       /* body frame */
  float body_inertia[ZB_NUM_BODIES][6];   /* about COM, body frame: xx yy zz xy xz yz */
  /* revolute joint k: X_{k+1} = X_k * T(jp_pos, jp_rot) * Rz(q_k) * T(jc_pos, jc_rot) */
  float joint_parent_pos[ZB_NUM_DOF][3];
  float joint_parent_rot[ZB_NUM_DOF][4];
  float joint_child_pos[ZB_NUM_DOF][3];
  float joint_child_rot[ZB_NUM_DOF][4];
  /* links (Isaac Lab body order) */
  int32_t link_body[ZB_NUM_LINKS];
  float link_pos[ZB_NUM_LINKS][3];        /* link frame in body frame */
  float link_rot[ZB_NUM_LINKS][4];
  float link_com[ZB_NUM_LINKS][3];        /* authored link COM, body frame */
  /* collision shape = convex hull of two circles: centre C, semi-axes E1, E2 (body frame) */
  float link_circle[ZB_NUM_LINKS][2][9];
  float link_sphere[ZB_NUM_LINKS][2][4];  /* round-1 inscribed spheres (unused since self collision
                                          * runs GJK on the link hull; kept for the ABI layout) */
  float link_bound[ZB_NUM_LINKS][4];      /* bounding sphere of the shape: centre (body), radius */
  int32_t num_self_pairs;
  int32_t self_pairs[ZB_MAX_SELF_PAIRS][2];
  /* defaults */
  float default_root_pos[3];
  float default_root_quat[4];
  float default_joint_pos[ZB_NUM_DOF];
  /* ImplicitActuatorCfg (zbot_cfg.py:658-668) + rigid props (zbot_cfg.py:626-634) */
  float kp, kd, effort_limit, velocity_limit, max_depenetration_velocity;
  /* RigidBodyPropertiesCfg.max_angular_velocity (zbot_cfg.py:632: 1000 deg/s, Isaac Lab's unit),
   * in rad/s: PhysX clamps the articulation root link's angular velocity to it */
  float max_angular_velocity;
  /* indices used by the MDP */
  int32_t base_link, foot_links[2], undesired_links[10];
  /* Isaac Lab's view when its articulation root is not chain link 0 (zbot_6s_v09.usd: the base):
   * the root link, its pose in the chain root's frame at the default joints, and per internal joint
   * k the Isaac Lab (breadth-first) joint index and sign (q_isaac = sign * q_internal) */
  int32_t api_root_link;
  float api_root_in_root[7];    /* pos 3, quat wxyz 4 */
  int32_t api_joint_index[ZB_NUM_DOF];
  float api_joint_sign[ZB_NUM_DOF];
  /* bit ci: circle ci of the link coincides with a circle of a lower link of the same composite
   * (the mated faces across a fixed joint); ground detection skips it (one contact set per face) */
  int32_t link_circle_dup[ZB_NUM_LINKS];
} zb_model;

/* Task / simulation constants: ZbotDirectEnvCfgV2 (v2.py:26-206) or Zbot6SUpEnvCfg
 * (standup.py:191-447) + solver parameters. Fields marked "standup" are ignored by the walking task. */
typedef struct zb_task_cfg {
  float sim_dt;                /* 1/200 (v2.py:48) */
  int32_t decimation;          /* 4 (v2.py:40) */
  int32_t max_episode_length;  /* ceil(20 s / 0.02 s) = 1000 (v2.py:39) */
  float termination_height;    /* 0.22 (v2.py:44) */
  float reward_scales[ZB_NUM_REWARD_TERMS]; /* walking: weights x step_dt (v2.py:250-252);
                                              standup: weights, the kernel multiplies by step_dt
                                              per term (standup.py:624) */
  float terminal_penalty;      /* 20 (v2.py:380); standup 2 (standup.py:630) */
  float joint_speed_limit;     /* 1.0 (v2.py:243) */
  float gravity;               /* 9.81 */
  float friction;              /* static friction 1.0, multiply combine (v2.py:49-56,62-68) */
  float contact_force_threshold; /* 1.0 N ContactSensorCfg.force_threshold default */
  float contact_margin;        /* speculative contact distance (m) */
  float baumgarte;             /* penetration correction per step (fraction) */
  int32_t solver_iterations;   /* PGS sweeps per substep */
  int32_t enable_self_collision;
  int32_t task;                /* ZB_TASK_* */
  /* standup / v4: reset_root_state_uniform pose ranges {lo, hi} of x, y, roll, yaw added to the
   * default root pose (standup.py:159-175, v4.py:274); pitch and z ranges are 0 there */
  float reset_pose_range[4][2];
  int32_t reset_pose_body_frame; /* 1: root quat * delta (v4.py:88), 0: delta * root quat (standup.py:88) */
  float center_z_init;         /* standup: center_z_last after a reset, 0.05 (standup.py:511,701) */
  float center_z_drop;         /* standup: died when center_z_last - base z > this, 0.05 (638) */
  int32_t center_z_period;     /* standup: center_z_last refresh when ep_len % period == period-1 (640) */
  /* standup / v4 my_curriculum (standup.py:99-111, v4.py:137-199): stage s >= 1 is entered at the
   * first call with resets once common_step_counter >= stage_steps[s], one stage per call */
  int32_t num_stages;          /* 1 = no curriculum */
  int32_t stage_steps[ZB_MAX_STAGES];
  float stage_scales[ZB_MAX_STAGES][ZB_MAX_REWARD_TERMS]; /* reward weights of each stage (x step_dt in-kernel) */
  float stage_prob_pos[ZB_MAX_STAGES]; /* v4: resample_commands prob_pos of each stage */
  /* v4 resample_commands (v4.py:107-135; reset and interval events 400-439) */
  float cmd_vel_range[2];      /* initial velocity_range (0.3, 0.3) */
  float cmd_yaw_range[2];      /* initial yaw_range (-0.1, 0.1) */
  int32_t cmd_dual_sign;
  float cmd_offset;
  float cmd_interval_s[2];     /* interval_range_s (3, 6) */
  /* v4 range_curriculum (v4.py:201-265, cfg 392-398 + 686) */
  float range_limit_vel[2], range_limit_yaw[2];
  int32_t range_start_steps;   /* max_episode_length * 48 */
  int32_t range_period_steps;  /* max_episode_length * 12 */
  int32_t range_min_buffer;    /* 20 */
  float range_threshold;       /* 0.85 */
  float range_delta;           /* 0.05 */
  float undesired_force_threshold; /* died: max |F| of an undesired body over the history > this (v2 1.0, v4 0.5) */
  float feet_f_last_init;      /* v4 feet_contact_forces_last after construction / reset: 15 (v4.py:731,979) */
  /* manager env (zbotlab_env_cfg.py): RelativeJointPositionAction, observation noise, command
   * term, terminations; the command ranges reuse cmd_vel_range (lin_vel_x) and cmd_yaw_range
   * (lin_vel_y), and lin_vel_cmd_levels reuses range_* (limit_ranges x / y, delta 0.1, threshold
   * 0.8, period max_episode_length; curriculums.py:57-83) */
  float action_scale;          /* 0.04 pi (zbotlab_env_cfg.py:125-131) */
  float action_clip;           /* processed-action clip +-0.04 pi */
  int32_t obs_corruption;      /* ObsGroup enable_corruption */
  float obs_noise[3];          /* additive U(-n, n): base quat 0.01, joint pos 0.01, joint vel 1.5 */
  float cmd_resample_s;        /* resampling_time_range (10, 10) */
  float cmd_rel_standing;      /* rel_standing_envs 0.02 */
  float feet_close_min;        /* feet_close termination: feet distance < 0.12 m */
  /* feet_down_pos_last on reset (v2.py:436, v4.py:996, mdp/rewards.py:42): 0 = the pre-reset
   * (terminal) feet positions, as the reference's call order reads them (body_link_pos_w before
   * DirectRLEnv.step's sim.forward()); 1 = the post-reset feet positions */
  int32_t reset_feet_refresh;
  /* dynamic (sliding) friction of the uniform-material tasks: 1.0 (v2.py:49-56,62-68); a contact
   * whose friction impulse would exceed mu_static * normal slides with mu_dynamic * normal */
  float friction_dynamic;
  /* contact solve per substep: 0 = solver_iterations projected Gauss-Seidel sweeps on one
   * linearisation (bias from the substep's initial separation); 1 = TGS-style (PhysX TGS,
   * zbot_cfg.py:637-638 solver_position_iteration_count 4 / velocity 0): solver_iterations
   * sub-iterations of h = sim_dt / solver_iterations, each one sweep whose contact biases are
   * re-linearised from the separation advanced by the normal velocities of the previous ones, the
   * pose integrated with the mean of the sub-iteration velocities; 2 = mode 1 plus
   * the per-position-iteration refresh of the ground contacts: before each sub-iteration after the
   * first, every ground contact's point (its rim candidate re-supported), separation and Jacobian
   * rows are re-evaluated at the pose the sub-iterations so far reached (walking v2 and stand-up) */
  int32_t solver_mode;
  /* self-contact manifold (PhysX PCM keeps up to 4 points per convex pair; zbot_cfg.py:636
   * enabled_self_collisions): 1 = a pair whose two nearest features are disk faces (cap on cap)
   * contributes up to 4 points (rim points of either face inside the other), every
   * other pair its one GJK point; 2 (default) = 1 plus side-by-side pairs whose nearest features are
   * two rulings within 5 degrees of the contact plane and of each other: the GJK point and the two
   * ends of the rulings' overlap (up to 3 points); 3 = 2 plus a ruling lying on a face (a face on one
   * side, a ruling within 5 degrees of the contact plane on the other): the GJK point and the ends of
   * the ruling's stretch over the face disk (up to 3 points; walking v2 and stand-up, whose kernels
   * for it are separate builds); a ruling-on-face pair that keeps no end point is tested as a
   * side-by-side pair as in 2 (a pair that qualifies for both takes the ruling-on-face points: 30 of
   * 56 side-by-side pairs in 200 k random folds, 3 of whose envs end with one point fewer than in
   * mode 2); 0 = one point per pair */
  int32_t self_manifold;
  /* walking v2: bit t set = reward term t is in the active reward_cfg (v2.py:246-257 builds
   * reward_functions from its keys). The reference updates a stateful term's buffers inside its
   * _reward_<name> only, so they advance only while the term is active: base_heading_x_sum
   * (v2.py:484-487), base_pos_y_err_sum (497-500), step_length's touchdown latches and
   * feet_contact_forces_last (509-533), feet_force_sum (567-571). A term can be active with
   * weight 0. Other tasks ignore it. zb_create rejects a walking-v2 cfg in which a term with a non-zero
   * reward_scales[t] has bit t clear (set every bit, 0xFFFFFFFF, for "all terms active").
   * ABI: this trailing field was added in round 5; a caller built against the older struct must be
   * rebuilt (sizeof(zb_task_cfg) grew by 4 bytes). */
  uint32_t reward_active;
} zb_task_cfg;

typedef struct zb_sim* zb_handle;

/* Create N envs on HIP device `hip_device`; state starts at the default pose, ep_len 0.
 * `seed` drives the full-reset episode_length_buf randomisation (v2.py:418-422). */
int zb_create(const zb_model* m, const zb_task_cfg* c, int num_envs, int hip_device, uint64_t seed,
              zb_handle* out);
void zb_destroy(zb_handle h);
const char* zb_last_error(void);
int zb_num_envs(zb_handle h);

/* Reset env_ids (device int32[n]); env_ids == NULL => all envs, which also draws
 * episode_length_buf ~ U{0..max_episode_length-1} (v2.py:418-422). */
int zb_reset(zb_handle h, const int32_t* env_ids, int n, void* stream);

/* One policy step for all envs. actions: device float[N][6] (raw policy output);
 * obs: device float[N][23] (standup: float[N][22]); reward: float[N]; terminated/truncated:
 * uint8[N] (torch.bool). */
int zb_step(zb_handle h, const float* actions, float* obs, float* reward, uint8_t* terminated,
            uint8_t* truncated, void* stream);

/* Observation of the current state (v2.py:351-365), as reset() returns. obs: float[N][23]. */
int zb_observe(zb_handle h, float* obs, void* stream);

/* Episode log of the most recent step with resets: term_means[ZB_LOG_LEN] (layout at
 * ZB_LOG_LEN; walking v2: mean episodic sum / 20 s, standup / v4: mean of sum / own duration),
 * counts[ZB_LOG_COUNTS] (layout at ZB_LOG_COUNTS; v2.py:441-459). Device pointers. */
int zb_read_log(zb_handle h, float* term_means, int32_t* counts, void* stream);
/* Register caller-owned device buffers (float[ZB_LOG_LEN], int32[ZB_LOG_COUNTS]) that every later step/reset with
 * resets fills in stream order, exactly as zb_read_log would (no per-step copies). NULL, NULL
 * unregisters. */
int zb_set_log_buffers(zb_handle h, float* term_means, int32_t* counts);
/* Register a caller-owned device accumulator float[ZB_LOG_LEN + ZB_LOG_COUNTS]: every later zb_step
 * adds the log's current values to it in stream order (the term means as zb_read_log returns them --
 * this step's when it had resets, else the last step-with-resets' -- then the counts as floats),
 * inside the step's finalize launch. It replaces the host runner's per-step sum of extras["log"]
 * (rsl_rl's OnPolicyRunner appends every step's log and averages it at log time,
 * rsl_rl/runners/on_policy_runner.py; the reference's train.py:205 runner.learn). Resets do not
 * add. NULL unregisters. */
int zb_set_log_accumulator(zb_handle h, float* acc);
/* Register a caller-owned device int64[N]: every later zb_step writes terminated | truncated into it
 * (rsl_rl's dones, RslRlVecEnvWrapper.step; isaaclab_rl's wrapper computes it with two torch ops per
 * step) from the step kernel's own flag stores. NULL unregisters. */
int zb_set_done_buffer(zb_handle h, int64_t* dones);

/* Persistent state, device float[zb_state_dim(h)][N] (ZB_STATE_DIM / ZB_SU_STATE_DIM).
 * zb_set_state also invalidates the contact cache below. */
int zb_state_dim(zb_handle h);
int zb_get_state(zb_handle h, float* dst, void* stream);
int zb_set_state(zb_handle h, const float* src, void* stream);

/* The solver's persistent self-contact cache (every task), device float[ZB_WARM_ROWS][N] ({normal,
 * code} of the first ZB_WARM_SLOTS kept self contacts of the last substep; code -1: none), the GJK
 * warm start of the next step's first substep. Simulator-internal like PhysX's contact cache (no
 * reference analogue: Isaac Lab never reads it); zb_set_state and resets invalidate it. Parity
 * tests copy it to the oracle for lock-step comparisons. */
int zb_get_contact_cache(zb_handle h, float* dst, void* stream);
int zb_set_contact_cache(zb_handle h, const float* src, void* stream);

/* Parity/debug: run `nsub` physics substeps with joint targets float[N][6] (no MDP);
 * if net_force != NULL it receives the last substep's net contact force, float[N][12][3],
 * and applied_torque (if != NULL) Isaac Lab's clipped PD estimate float[N][6]. The persistent
 * self-contact cache is invalidated (the next zb_step's first substep starts GJK cold). */
int zb_physics_substeps(zb_handle h, const float* targets, int nsub, float* net_force,
                        float* applied_torque, void* stream);

/* Standup / manager: per-link friction coefficients, device float[N][12] (link order of
 * ZB_NUM_LINKS), e.g. the static / dynamic friction sampled by randomize_rigid_body_material
 * (standup.py:124-136). Ground contacts use mu[link] * cfg.friction (the terrain's coefficient,
 * multiply combine), self contacts mu[a] * mu[b], for the static and the dynamic coefficient
 * alike. A new handle starts at cfg.friction / cfg.friction_dynamic for every link.
 * zb_set_link_friction sets both coefficients to `mu`; zb_set_link_friction_sd sets them apart. */
int zb_set_link_friction(zb_handle h, const float* mu, void* stream);
int zb_set_link_friction_sd(zb_handle h, const float* mu_static, const float* mu_dynamic, void* stream);

/* Curriculum stage and common_step_counter (zb_step calls). Host pointers; synchronises. */
int zb_read_curriculum(zb_handle h, int32_t* stage, int64_t* common_step_counter);

/* Measurement: time the next `max_launches` zb_step_kernel launches with hipEvents recorded on
 * the launch stream right around the kernel (bench.py's roofline figure). zb_profile_end waits
 * for the last event and returns the summed kernel time. */
int zb_profile_begin(zb_handle h, int max_launches);
/* Time only every stride-th zb_step launch from now on (default 1): the event-recording dispatch
 * adds ~5.7 us to the step it brackets (bench.py samples every 8th timed step). */
int zb_profile_stride(zb_handle h, int stride);
int zb_profile_end(zb_handle h, float* total_ms, int* count);

/* Diagnostic builds only (compiled with -DZB_STAMPS): per-phase s_memtime cycle sums of
 * zb_step_kernel over all waves since the previous call (phases: DESIGN.md §7). Returns <0 in
 * the product build. */
int zb_read_stamps(uint64_t* out16);
/* diagnostic build only: the phase cycles of the slowest wave (same order as zb_read_stamps) */
int zb_read_stamps_slowest(uint64_t* out16);
/* diagnostic build only: per-launch wave histograms since the previous call: [0, 64) the wave's
 * largest count of GJK pairs of one env in one substep, [64, 128) the wave's largest per-lane sum
 * of GJK iterations over the step (bins of 4); [128, 136) contact-cap counters over env-substeps:
 * env-substeps, more than ZB_MAX_CONTACTS candidates, more than 18 self contacts, self contacts on
 * overlapping cores, env-substeps with one, self contacts, ground candidates */
int zb_read_stamp_hist(uint64_t* out136);
/* Diagnostic build only: per workgroup of the latest step launch, 23 values {start, end
 * (s_memrealtime, 100 MHz), 13 phase cycle counts, 8 substep end times (walking v2)}; out [n][23]. */
int zb_read_wave_times(uint64_t* out, int n);

/* Test entry: the self-collision GJK (the step kernels' gjk_quad) on n link pairs given as
 * world-frame core hulls, device pointers. pairs [n][2][2][9] (per hull two circles: centre, E1,
 * E2 with the radius baked in), v0 [n][3] start directions or NULL (the hull centre difference),
 * out [n][9] = {contact, separation, normal[3], point[3], iterations}. Checked against the
 * oracle's hull_pair (tests/test_gpu_selfcollision.py). */
int zb_gjk_pairs(const float* pairs, const float* v0, int n, float margin, float* out, void* stream);

/* Test entry: GJK (cold start) + the self-contact face manifold (the step kernels' quad_manifold,
 * zb_task_cfg.self_manifold) on n link pairs given as world-frame core hulls (layout as
 * zb_gjk_pairs); out [n][29] = {points (0: no contact, 1: the GJK contact alone), then per point
 * {separation, normal[3], point[3]}}. Checked against the oracle's zbo_pair_manifold. */
int zb_pair_manifold(const float* pairs, int n, float margin, float* out, void* stream);
/* The same with the manifold mode (zb_task_cfg.self_manifold 1..3; zb_pair_manifold = mode 2). */
int zb_pair_manifold_mode(const float* pairs, int n, float margin, int mode, float* out, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* ZBOT_H_ */
