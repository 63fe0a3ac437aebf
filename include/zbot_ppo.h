/*
 * zbot_ppo.h — C ABI of libzbot_ppo.so: the PPO minibatch update of the rsl_rl ActorCritic on
 * MI355X as hand-written fp32 MFMA kernels (zbot_lab_amd/csrc/ppo_mlp.hip).
 *
 * Replaces, per minibatch of PPO.update (reference: rsl_rl's PPO as configured by
 * source/zbot/zbot/tasks/zbot6b_direct/agents/rsl_rl_ppo_cfg.py:65-91 and walked through in
 * ppo_learning_notes.md:521-548; restated in zbot_lab_amd/rl/ppo.py:PPO.update_steps):
 *   policy.update_distribution(obs_b) -> log_prob / evaluate(critic_obs_b) / entropy -> adaptive-KL
 *   statistic -> clipped surrogate + clipped value loss - entropy bonus -> loss.backward()
 * i.e. the actor and critic MLP forward passes, the loss and its gradient, and the backward pass
 * into every parameter's .grad (weights, biases, the Gaussian std). Gradient averaging across
 * ranks, the learning-rate rule, gradient clipping and Adam stay with the caller (torch), or run
 * fused in zbp_optimizer_step on one GPU.
 *
 * All pointers are device pointers (torch tensors' data_ptr), fp32 unless stated; every call is
 * ordered on `stream` (a hipStream_t) and never synchronises the host, so a sequence of calls can
 * be captured in a HIP graph. Returns 0 on success, a negative code on a bad argument or a HIP
 * error (zbp_last_error() describes it).
 */
#ifndef ZBOT_PPO_H
#define ZBOT_PPO_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZBP_MAX_LAYERS 4 /* linear layers per MLP (3 hidden + output, the rsl_rl cfgs here) */

/* One MLP (torch nn.Sequential of Linear / ELU): layer l maps dim[l] -> dim[l+1]; ELU after every
 * layer but the last. Limits: dim[0] <= 32 (observations), hidden dims multiples of 32 up to 256,
 * output dim <= 32. */
typedef struct {
  int32_t n_layers;
  int32_t dim[ZBP_MAX_LAYERS + 1];
  const float* w[ZBP_MAX_LAYERS]; /* Linear.weight [dim[l+1]][dim[l]] (row-major, contiguous) */
  const float* b[ZBP_MAX_LAYERS]; /* Linear.bias [dim[l+1]] */
  float* gw[ZBP_MAX_LAYERS];      /* their .grad buffers (overwritten by zbp_minibatch) */
  float* gb[ZBP_MAX_LAYERS];
} zbp_net;

/* The rollout (RolloutStorage, flattened [T * N] rows) and this minibatch's rows:
 * rows idx[idx_offset .. idx_offset + batch) of the permutation (int64, rsl_rl's randperm). */
typedef struct {
  const float* obs;          /* [rows][obs_dim] */
  const float* critic_obs;   /* [rows][critic_obs_dim] */
  const float* actions;      /* [rows][num_actions] */
  const float* values;       /* [rows] target values */
  const float* advantages;   /* [rows] */
  const float* returns;      /* [rows] */
  const float* log_prob;     /* [rows] old log-probabilities */
  const float* mu;           /* [rows][num_actions] old action means */
  const float* sigma;        /* [rows][num_actions] old action stds */
  const int64_t* idx;        /* the update's permutation */
  int64_t idx_offset;
  int32_t batch;             /* minibatch rows (a multiple of 32) */
  int32_t obs_dim, critic_obs_dim, num_actions;
} zbp_batch;

/* PPO loss constants (RslRlPpoAlgorithmCfg) */
typedef struct {
  float clip_param, value_loss_coef, entropy_coef;
  int32_t use_clipped_value_loss;
} zbp_loss_cfg;

/* Workspace floats for nets of these shapes and minibatch size (the caller allocates one float
 * buffer of that size, 256-byte aligned, and passes it to every call). */
int64_t zbp_workspace_floats(const zbp_net* actor, const zbp_net* critic, int32_t batch);

/* Copy the current parameters into the workspace's padded / transposed images. Call once before
 * the first zbp_minibatch of an update and after every parameter change made outside
 * zbp_optimizer_step (a torch optimizer step, a checkpoint load). */
int zbp_pack(const zbp_net* actor, const zbp_net* critic, float* ws, int32_t batch, void* stream);

/* One minibatch: forward, loss, backward. Writes every .grad of both nets and std_grad
 * [num_actions], and stats[4] = {kl_mean, value_loss, surrogate_loss, entropy_mean} of the
 * minibatch (the KL statistic of the adaptive learning-rate rule and the loss terms). */
int zbp_minibatch(const zbp_net* actor, const zbp_net* critic, const float* std_param, float* std_grad,
                  const zbp_batch* batch, const zbp_loss_cfg* loss, float* ws, float* stats, void* stream);

/* Adam (torch.optim.Adam semantics, betas b1 / b2, eps, no weight decay) fused with rsl_rl's
 * adaptive learning-rate rule and global-norm gradient clipping, for one GPU:
 *   lr <- adaptive(lr, stats[0]) (desired_kl > 0; lr / 1.5 above 2 desired_kl, x 1.5 below half of
 *   it, within [1e-5, 1e-2]); grads scaled by min(1, max_norm / (||g|| + 1e-6)); step += 1;
 *   m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2; p -= lr / (1 - b1^t) * m / (sqrt(v) / sqrt(1 - b2^t) + eps)
 * over the params listed in `params` (the torch optimizer's param order): n_params tensors with
 * numel / param / grad / exp_avg / exp_avg_sq pointers. lr and step are device scalars (torch's
 * capturable Adam keeps `step` as a float tensor; one shared step counter is read from step[0] and
 * every tensor's own counter written). Then re-packs the workspace (zbp_pack). acc[3] += stats[1..3].
 * norm_from_minibatch != 0: the gradient norm comes from the per-tile sums of squares the last
 * zbp_minibatch on this workspace left (one launch fewer); only valid when the .grad buffers and
 * std_grad are still exactly what that call wrote (one GPU, no all-reduce or hook in between);
 * 0: recomputed from params->grad. */
#define ZBP_MAX_PARAMS 24
typedef struct {
  int32_t n_params;
  int64_t numel[ZBP_MAX_PARAMS];
  float* param[ZBP_MAX_PARAMS];
  float* grad[ZBP_MAX_PARAMS];
  float* exp_avg[ZBP_MAX_PARAMS];
  float* exp_avg_sq[ZBP_MAX_PARAMS];
  float* step[ZBP_MAX_PARAMS];
} zbp_params;
int zbp_optimizer_step(const zbp_params* params, float* lr, const float* stats, float* acc, float desired_kl,
                       float max_grad_norm, float beta1, float beta2, float eps, const zbp_net* actor,
                       const zbp_net* critic, float* ws, int32_t batch, int32_t norm_from_minibatch,
                       void* stream);

/* GAE (RolloutStorage.compute_returns): rewards / dones / values [steps][envs] (time-out bootstrap
 * already in the rewards), last_values [envs] -> returns, advantages = returns - values, then (if
 * normalize) advantages normalised by their mean and unbiased std (+1e-8). scratch: >= 258 floats. */
int zbp_gae(const float* rewards, const float* dones, const float* values, const float* last_values, float* returns,
            float* advantages, int32_t steps, int32_t envs, float gamma, float lam, int32_t normalize, float* scratch,
            void* stream);

/* One rollout step of PPO.act (rsl_rl ActorCritic.act / evaluate / get_actions_log_prob and the
 * transition fields of RolloutStorage.add; zbot_lab_amd/rl/ppo.py) for `rows` envs in one launch:
 * actions = mu + std * noise (noise: the caller's standard-normal draw, [rows][num_actions], or NULL:
 * drawn in the kernel, a counter-based standard normal keyed by noise_seed, the workspace's draw
 * counter -- which every zbp_pack / zbp_optimizer_step advances --, noise_step, the row and the
 * action), its
 * Gaussian log-probability summed over the actions, the critic's value; writes actions [rows][na]
 * (the env's input) and the storage slot of this step: observations, critic observations, actions,
 * values, log-probabilities, mu, sigma. Reads the workspace's weight images (zbp_pack must follow
 * every parameter change; zbp_optimizer_step re-packs itself). Replaces the ~30 torch kernels of a
 * policy step (runner._rollout). */
typedef struct {
  const float* obs;         /* [rows][obs_dim] */
  const float* critic_obs;  /* [rows][critic_obs_dim] */
  const float* noise;       /* [rows][num_actions], or NULL (in-kernel draw) */
  float* actions;           /* [rows][num_actions] out */
  float* st_obs;            /* storage slot [rows][obs_dim] out */
  float* st_critic_obs;     /* [rows][critic_obs_dim] out */
  float* st_actions;        /* [rows][num_actions] out */
  float* st_values;         /* [rows] out */
  float* st_log_prob;       /* [rows] out */
  float* st_mu;             /* [rows][num_actions] out */
  float* st_sigma;          /* [rows][num_actions] out */
  int32_t rows, obs_dim, critic_obs_dim, num_actions;
  int32_t noise_step;       /* (noise == NULL) the rollout step: distinct draws per step of a rollout */
  int32_t noise_seed;       /* (noise == NULL) the caller's stream, e.g. one per rank */
} zbp_act_io;
int zbp_act(const zbp_net* actor, const zbp_net* critic, const float* std_param, const zbp_act_io* io, float* ws,
            int32_t batch, void* stream);
/* PPO.process_env_step + the runner's episode statistics for one step (runner._rollout): storage
 * reward = reward (+ gamma * value where time_outs, rsl_rl's bootstrap; time_outs may be NULL),
 * storage done = done; cur_rew += reward, cur_len += 1, and over the envs with done > 0
 * ep_stats[0..2] += {sum cur_rew, sum cur_len, count} before their cur_rew / cur_len reset to 0.
 * rewards / values / cur_* [n] fp32, dones [n] int64, time_outs [n] uint8 (bool). One launch. */
int zbp_env_post(const float* rewards, const int64_t* dones, const uint8_t* time_outs, const float* values, float gamma,
                 float* st_rewards, float* st_dones, float* cur_rew, float* cur_len, float* ep_stats, int32_t n,
                 void* stream);
const char* zbp_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* ZBOT_PPO_H */
