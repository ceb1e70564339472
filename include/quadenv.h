/*
 * quadenv.h -- C ABI of libquadenv.so, the MI355X-native vectorized quadrotor env.
 *
 * This is the drop-in boundary for the reference's hot path: N independent copies of
 *   HoverEnv.step / HoverEnv.reset                 (envs/hover_env.py:159-198, :200-238)
 *   RateControlWrapper.action / .step / .reset      (envs/rate_wrapper.py:69-111)
 *   TrajectoryFollowEnv.step / .reset               (envs/trajectory_follow_env.py:145-174,
 *                                                    :220-253)
 * including the mujoco.mj_step they call (hover_env.py:180) and the SB3 VecEnv auto-reset
 * around them (train.py:48, DummyVecEnv semantics), executed as HIP kernels on gfx950 over a
 * struct-of-arrays batch resident in HBM.
 *
 * Conventions
 *  - Plain C types only; `void* stream` is a hipStream_t (e.g. torch.cuda.current_stream()
 *    .cuda_stream); NULL = the legacy default stream. Every call that launches work enqueues it
 *    on that stream and returns without synchronizing (graph-capturable), except get/set_state
 *    with host pointers, which synchronize the stream.
 *  - Device pointers are caller-owned (torch tensors' data_ptr()); the handle owns only the env
 *    state. Row-major shapes are given as [rows, cols].
 *  - Return 0 on success, a negative QUAD_E* code on error; the message is available from
 *    quad_last_error() (thread-local). Nothing aborts or throws across the ABI.
 *  - A handle is bound to one device and is not internally locked (one handle per process per
 *    GPU; multi-GPU = one process per GPU with disjoint env_id_base ranges).
 */
#ifndef QUADENV_H
#define QUADENV_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QUADENV_ABI_VERSION 5

enum { QUAD_OK = 0, QUAD_EINVAL = -1, QUAD_EHIP = -2, QUAD_ENOMEM = -3, QUAD_EMODEL = -4 };
/* QUAD_ENV_BRAX_HOVER / QUAD_ENV_BRAX_TRAJ: the brax Env API siblings of the same path
 * (train_brax_ppo.py QuadHoverBraxEnv :39-176 / JaxMJXQuadBraxEnv :179-368) as brax's ppo.train
 * wraps them (EpisodeWrapper truncation, AutoResetWrapper restoring the episode's first state):
 * 21-D raw obs [qpos(11), qvel(10)], clipped physical action -> mixer (no voltage), mjx.step
 * semantics (no MuJoCo-C bad-state resets). */
enum { QUAD_ENV_HOVER = 0, QUAD_ENV_TRAJ = 1, QUAD_ENV_BRAX_HOVER = 2, QUAD_ENV_BRAX_TRAJ = 3 };
/* QUAD_WRAP_RELPOS: RelPosActWrapper (envs/wrappers.py:13-25): 7-D obs [normalized rel pos (3),
 * previous action (4)] of the hover / trajectory kinds (quad_step's obs is then [N,7]).
 * QUAD_WRAP_CTBR_RELPOS: the stack the reference README documents,
 * RelPosActWrapper(RateControlWrapper(env)): the CTBR controller maps the rate action to torques
 * (rate_wrapper.py:69-98) and the 7-D obs carries the RATE action as the previous action
 * (rate_wrapper.py:100-106 overwrites unwrapped._prev_action after the base step). */
enum { QUAD_WRAP_NONE = 0, QUAD_WRAP_CTBR = 1, QUAD_WRAP_RELPOS = 2, QUAD_WRAP_CTBR_RELPOS = 3 };
enum { QUAD_NQ = 11, QUAD_NV = 10, QUAD_OBS = 12, QUAD_OBS_BRAX = 21, QUAD_OBS_RELPOS = 7, QUAD_ACT = 4 };

/* Env configuration. quad_default_cfg() fills the reference's defaults:
 *  HoverEnv.__init__ (hover_env.py:15-100), TrajectoryFollowEnv.__init__
 *  (trajectory_follow_env.py:22-104), RateControlWrapper.__init__ (rate_wrapper.py:40-64) with
 *  pid_gains.json:43-52, drone_config.py:9-22, drone.xml:4 (timestep, gravity, fluid). */
typedef struct QuadCfg {
  int32_t env_kind;          /* QUAD_ENV_HOVER | QUAD_ENV_TRAJ */
  int32_t wrapper;           /* QUAD_WRAP_NONE | _CTBR (RateControlWrapper) | _RELPOS | _CTBR_RELPOS */
  int32_t max_episode_steps; /* 512 hover / 2048 traj */
  int32_t auto_reset;        /* 1: SB3 VecEnv semantics (reset on terminated|truncated) */
  float obs_low[12], obs_high[12];       /* HoverEnv._obs_bounds   (normalization) */
  float init_low[12], init_high[12];     /* HoverEnv._initial_state_bounds */
  float target_low[3], target_high[3];   /* HoverEnv._target_pos_bounds (hover only) */
  float term_low[12], term_high[12];     /* HoverEnv._state_bounds (termination) */
  float act_low[4], act_high[4];         /* HoverEnv._action_bounds */
  double max_motor_thrust, arm_length, yaw_coeff; /* max_motor_thrust: finite, >= 0 (else QUAD_EINVAL) */
  double nominal_voltage, min_voltage, vdrop_base, vdrop_load;
  double rate_max_rad, rate_kd[3], rate_ki, rate_imax, inertia[3], max_torque;
  double timestep, gravity[3], density, viscosity;
  /* brax kinds only (train_brax_ppo.py): target = target_low (QuadHoverBraxEnv (0,0,1));
   * position limits = term_low/high[0..2] (|x|,|y| <= 3, z in [0.02, 4]); act_low/high = the
   * clip range of the physical action; max_episode_steps = --episode-length (500). */
  float reset_noise;            /* U(+-noise) on qpos and qvel at reset (0.01) */
  float reward_pos_coef;        /* exp(-coef |pos - target|^2): 2 hover, 1 jax_mjx */
  float reward_action_coef;     /* - coef |a|^2 (jax_mjx 0.001) */
  float vel_limit;              /* jax_mjx: any |v_i| > limit invalidates (20) */
  float traj_center[3], traj_amp[3], traj_freq[3];  /* jax_mjx sinusoid target */
  float traj_duration;          /* seconds spanned by the episode_length samples (5) */
  /* TrajectoryFollowEnv's info-only spline (trajectory_follow_env.py:175-243): center ~
   * U(spline_center_low, _high), n_wp ~ {3,4,5}, offsets ~ U(+-spline_amp), first waypoint = start
   * position, natural cubic spline sampled at max_episode_steps points over spline_duration s. */
  float spline_center_low[3], spline_center_high[3], spline_amp[3];
  float spline_duration;        /* 30 */
} QuadCfg;

/* Env state in field-major SoA: each array is [fields][N] (qpos [11][N], qvel [10][N], ...).
 * qpos = MuJoCo qpos (x y z qw qx qy qz theta1..4), qvel = MuJoCo qvel (world v, body omega,
 * prop rates); voltage = HoverEnv.voltage; target = target_state.position; rate_int =
 * RateControlWrapper._rate_int_torque; step_count = HoverEnv._step_count; episode = the number of
 * resets drawn so far (the reset RNG counter); prev_action = HoverEnv._prev_action [4][N] (kept for
 * QUAD_WRAP_RELPOS). NULL members are skipped by get/set. */
typedef struct QuadStateSoA {
  float* qpos;
  float* qvel;
  float* voltage;
  float* target;
  float* rate_int;
  int32_t* step_count;
  uint32_t* episode;
  float* prev_action;
} QuadStateSoA;

/* Outputs of quad_step (device pointers). Required: obs, reward, terminated, truncated.
 *  obs            [N,12] normalized observation (after auto-reset for envs that finished);
 *                        brax kinds: [N,21] raw [qpos, qvel]
 *  reward         [N]    exp(-|pos - target|^2)           (hover_env.py:138-141)
 *  terminated     [N]    NaN / state-bounds termination   (hover_env.py:150-157)
 *  truncated      [N]    step_count >= max_episode_steps  (hover_env.py:188)
 * Optional (NULL to skip):
 *  terminal_obs   [N,12|21] obs before auto-reset (SB3 info["terminal_observation"]); only rows of
 *                        envs that finished this step are written
 *  motor_commands [N,4]  info["motor_commands"] (N)
 *  voltage_scale  [N]    info["voltage_scale"]
 *  state12        [N,12] info["state"]: absolute 12-D QuadState before auto-reset
 *  target_info    [N,9]  info["target"], ["target_vel"], ["target_acc"] before auto-reset: the
 *                        TrajectoryFollowEnv spline sample at min(step - 1, L - 1)
 *                        (trajectory_follow_env.py:163-168; regenerated from the episode's reset
 *                        draw, so it follows quad_reset/auto-reset episodes, not injected states);
 *                        the fixed target and zeros for the hover kinds */
typedef struct QuadStepOut {
  float* obs;
  float* reward;
  uint8_t* terminated;
  uint8_t* truncated;
  float* terminal_obs;
  float* motor_commands;
  float* voltage_scale;
  float* state12;
  float* target_info;
} QuadStepOut;

typedef struct QuadHandle QuadHandle;

int quad_abi_version(void);
const char* quad_last_error(void);

/* Fill `cfg` with the reference defaults for (env_kind, wrapper); auto_reset = 1. */
int quad_default_cfg(int32_t env_kind, int32_t wrapper, QuadCfg* cfg);

/* Allocate N envs on `device`. Global env ids are env_id_base .. env_id_base+N-1; the reset RNG
 * is Philox4x32-10 keyed by `seed` with counter (global env id, episode, draw block), so a
 * shard's trajectories do not depend on how many GPUs the envs are spread over.
 * State starts zeroed; call quad_reset before stepping. 1 <= N <= 33,554,431 (the state SoA is
 * addressed as one 4 GiB buffer resource); QUAD_EINVAL otherwise. */
int quad_create(const QuadCfg* cfg, int32_t device, uint64_t seed, uint64_t env_id_base,
                int32_t n_envs, QuadHandle** out);
void quad_destroy(QuadHandle* h);
int32_t quad_num_envs(const QuadHandle* h);
/* Diagnostics: the step-kernel form quad_create chose -- bit 4 set when the handle's constant block
 * is a reference default and the kernels with compiled-in constants run (QUADENV_SPEC=0 turns that
 * off), bit 5 always set for the hover / trajectory kinds (one thread per env with helper waves
 * drawing the resets, k_step_h; bits 0-3 were the lane-group forms removed in round 6), bit 7 set when those helper blocks are 256 envs wide (full-batch steps of 32,769 .. 2,097,151 envs,
 * or QUADENV_HBLOCK=256; 64-env blocks otherwise), bit 8 set when a full-batch step of those blocks
 * moves the env state with the nt cache policy (65,536-env-scale and >= 2M-env batches; QUADENV_NT
 * pins it), bit 9 set when those 64-env nt launches run as k_step_hd, the DRAM form with a
 * 7-waves-per-SIMD register budget (>= 4M-env batches; QUADENV_HD pins it). 64 alone: a RELPOS or brax handle, whose one step kernel (k_step_relpos / k_step_brax) has no forms. */
int32_t quad_kernel_form(const QuadHandle* h);

/* Re-key the reset RNG (HoverEnv.reset(seed=...), hover_env.py:210 -> gymnasium seeding) and
 * zero every env's episode counter (stream-ordered). */
int quad_seed(QuadHandle* h, uint64_t seed, void* stream);

/* HoverEnv.reset for every env (mask == NULL) or for envs with mask[i] != 0 (device [N] u8).
 * Writes the reset observation rows to obs (device [N,12]) when obs != NULL. */
int quad_reset(QuadHandle* h, const uint8_t* mask, float* obs, void* stream);

/* One vectorized env step: actions is device [N,4] float32 in the policy's normalized space
 * (the CTBR wrapper's rate space when wrapper == QUAD_WRAP_CTBR). Not clipped by the env. */
int quad_step(QuadHandle* h, const float* actions, const QuadStepOut* out, void* stream);

/* quad_step restricted to envs [first, first + count): rows of actions/out outside the range are
 * neither read nor written. Sub-ranges on different streams let independent halves of a batch
 * overlap (one half's physics with the other half's memory traffic, or with a policy kernel). */
int quad_step_range(QuadHandle* h, int32_t first, int32_t count, const float* actions,
                    const QuadStepOut* out, void* stream);

/* Measurement only (no reference counterpart; bench.py's live DRAM floor): the HBM traffic of one
 * quad_step with no compute -- the same env tiles, actions and output rows, with quad_step's cache
 * policy for this batch size: every env's 26 state words (qpos 11, qvel 10, voltage, target 3, step
 * counter) read and written back unchanged, its action read, and obs [N,12], reward, terminated and
 * truncated written (obs = the first 12 state words, reward = qpos[0], flags = 0). 278 bytes per env,
 * quad_step's algorithmic bytes. The env state is left as it was; the output rows are overwritten.
 * Hover / trajectory kinds without RELPOS. */
int quad_mem_floor(QuadHandle* h, const float* actions, const QuadStepOut* out, void* stream);

/* HoverEnv._get_obs for the current state (e.g. after quad_set_state). obs: device [N,12];
 * state12 (device [N,12] or NULL): the absolute QuadState vector (HoverEnv._state.vec()). */
int quad_observe(QuadHandle* h, float* obs, float* state12, void* stream);

/* Config 2 of the scope table -- the random-action rollout of debug_training.py:111
 * (env.step(env.action_space.sample()) in a loop) -- as ONE launch: `steps` consecutive quad_step
 * calls with the actions quad_random_actions(step0 + s) gives, the env state kept on chip between
 * steps. Results are identical to quad_random_actions + quad_step, step by step. Every QuadStepOut
 * pointer is time-major: obs [steps][N,12], reward / terminated / truncated [steps][N], terminal_obs
 * [steps][N,12] (optional; rows of envs that finished that step); motor_commands, voltage_scale,
 * state12 and target_info must be NULL. actions_out: [steps][N,4] (16-byte aligned) or NULL.
 * Hover / trajectory kinds, wrapper NONE or CTBR; steps * N * 48 < 2^32. */
int quad_step_random(QuadHandle* h, uint32_t step0, int32_t steps, const QuadStepOut* out, float* actions_out,
                     void* stream);

/* HoverEnv._is_terminated (hover_env.py:150-157; TrajectoryFollowEnv's bounds for that kind) on n
 * caller-given absolute 12-D states (device [n,12], the QuadState vector: pos, roll/pitch/yaw, world
 * velocity, body rates): terminated[i] = any non-finite component or any component outside the
 * handle's inclusive termination bounds -- the predicate quad_step applies after each step.
 * terminated: device [n] u8. Not defined for the brax kinds (QUAD_EINVAL). */
int quad_terminated(QuadHandle* h, const float* state12, int32_t n, uint8_t* terminated, void* stream);

/* action_space.sample() equivalent for synthetic rollouts: U[-1,1)^4 per env from
 * Philox(seed, global env id, step_index). actions: device [N,4]. */
int quad_random_actions(QuadHandle* h, uint32_t step_index, float* actions, void* stream);

/* Copy the env state out of / into the handle. `on_host` != 0: the SoA arrays are host memory
 * (the call synchronizes `stream`); otherwise device memory (async). */
int quad_get_state(QuadHandle* h, const QuadStateSoA* dst, int32_t on_host, void* stream);
int quad_set_state(QuadHandle* h, const QuadStateSoA* src, int32_t on_host, void* stream);

/* ---- Batched waypoint-following evaluation (row f4): evaluate.py:440-612 evaluate_trajectory
 * for N envs at once (hover / trajectory kinds, any wrapper). Waypoint sets are float64 (the
 * generators' numpy arrays) [n_sets][max_points][3]; env i follows set set_of[i] (0 if NULL). */
typedef struct QuadWaypoints {
  const double* points;    /* device [n_sets][max_points][3] */
  const int32_t* counts;   /* device [n_sets], >= 1 */
  const int32_t* set_of;   /* device [N] or NULL */
  int32_t max_points;
  float reach_radius;      /* --reach-radius (0.25) */
} QuadWaypoints;
/* Per-env tracker (device [N] arrays). status: 0 running, 1 lap completed, 2 terminated,
 * 3 truncated (max steps). */
typedef struct QuadWaypointState {
  int32_t* wp_idx;
  int32_t* reached;
  int32_t* laps;
  int32_t* steps;
  int32_t* status;
  double* total_reward;
} QuadWaypointState;
/* Start every env at its first waypoint (evaluate.py:487-505): qpos[0:7] = (wp0, 1, 0, 0, 0),
 * qvel[0:6] = 0 (props keep their reset state), target = wp[1 % n], rate integrator 0, step 0;
 * tracker zeroed with wp_idx = 1 % n; writes the observation (HoverEnv._get_obs, or the
 * RelPosActWrapper observation) to obs. Call after quad_reset. */
int quad_waypoints_begin(QuadHandle* h, const QuadWaypoints* w, const QuadWaypointState* s, float* obs,
                         void* stream);
/* After each quad_step (create the handle with auto_reset = 0): for envs still running, add the
 * reward, count the step, switch to the next waypoint when |pos - wp| < reach_radius (pos =
 * the step's state12[:, 0:3], info["state"]); completing the lap, terminated or truncated end
 * the env's evaluation (evaluate.py:545-595). The next waypoint is written as the env target. */
int quad_waypoints_update(QuadHandle* h, const QuadWaypoints* w, const QuadWaypointState* s,
                          const float* state12, const float* reward, const uint8_t* terminated,
                          const uint8_t* truncated, void* stream);

/* PPO rollout support (row P of the scope table): generalized advantage estimation over a
 * time-major rollout, SB3 RolloutBuffer.compute_returns_and_advantage semantics.
 *  rewards, values, episode_starts: device [T,N] float32 (episode_starts 1.0 where the step
 *  began a new episode); last_values [N]; dones [N] (1.0 if the env finished at the last step).
 *  Writes advantages and returns (= advantages + values), device [T,N]. */
int quad_gae(const float* rewards, const float* values, const float* episode_starts,
             const float* last_values, const float* dones, int32_t T, int32_t N, float gamma,
             float gae_lambda, float* advantages, float* returns, void* stream);

/* ---- Rollout policy on MFMA (row P): the SB3 ActorCritic that train.py:50-68 configures
 * (MlpPolicy, net_arch pi=[128,128] vf=[128,128], ReLU, state-independent log_std), fp32.
 * Parameter pointers are device fp32 in torch's nn.Linear layout ([out, in] row-major). */
typedef struct QuadPolicyParams {
  const float *pi_w0, *pi_b0, *pi_w1, *pi_b1;  /* mlp_extractor.policy_net.{0,2} [128,12] [128,128] */
  const float *act_w, *act_b;                  /* action_net [4,128] [4] */
  const float *vf_w0, *vf_b0, *vf_w1, *vf_b1;  /* mlp_extractor.value_net.{0,2} */
  const float *val_w, *val_b;                  /* value_net [1,128] [1] */
  const float* log_std;                        /* [4] */
} QuadPolicyParams;

/* Size (floats) of the packed policy image quad_policy_pack writes. */
int32_t quad_policy_packed_floats(void);

/* Repack the parameters into the MFMA fragment order the policy kernels read (call after every
 * optimizer update that precedes a rollout; stream-ordered). `packed`: device, 16-byte aligned. */
int quad_policy_pack(const QuadPolicyParams* p, float* packed, void* stream);

/* Rollout epilogue of one step (after quad_step), SB3 collect_rollouts semantics:
 * buf_rew[row] = reward + gamma * V(terminal_obs) where truncated && !terminated (TimeLimit
 * bootstrap; the critic runs only on 32-env tiles that hold such an env), else reward;
 * last_start = terminated | truncated; Monitor statistics: ep_ret/ep_len accumulate and reset on
 * done, stats[slot] += (finished return, length, 1) -- sum the QUAD_POLICY_STAT_SLOTS slots. */
enum { QUAD_POLICY_STAT_SLOTS = 1024 };
typedef struct QuadRolloutPost {
  const float* reward;          /* [N] */
  const uint8_t* terminated;    /* [N] */
  const uint8_t* truncated;     /* [N] */
  const float* terminal_obs;    /* [N,12] */
  float* buf_rew;               /* [rows,N] */
  float* last_start;            /* [N] */
  float* ep_ret;                /* [N] running episode return */
  float* ep_len;                /* [N] running episode length */
  double* stats;                /* [QUAD_POLICY_STAT_SLOTS][3], zeroed by the caller */
  int32_t rows;
  float gamma;
} QuadRolloutPost;

/* One rollout-step policy evaluation (SB3 OnPolicyAlgorithm.collect_rollouts body):
 * a = mean(obs) + exp(log_std) * z, z ~ N(0,1) from Philox(seed; env id, t, 0x200) + Box-Muller;
 * actions_env = clip(a, -1, 1). `cursor` (device uint32[4] = {t, pending, 0, 0}, zero it to start)
 * holds the running step counter t (never reset, so successive rollouts draw fresh noise); row
 * outputs go to row t % rows of time-major [rows,N,...] buffers; every row pointer may be NULL.
 * With `epilogue` != NULL the launch first finishes step t-1 if it is pending (QuadRolloutPost
 * above, row (t-1) % rows, before episode_starts[t] is taken from last_start), then advances the
 * cursor to t+1 and marks step t pending: one launch per step besides quad_step. */
typedef struct QuadPolicyAct {
  const float* obs;         /* [N,12] */
  float* actions_env;       /* [N,4] clipped action for quad_step (16-byte aligned) */
  float* actions;           /* [rows,N,4] unclipped sample (rollout buffer) or NULL */
  float* log_prob;          /* [rows,N] or NULL */
  float* value;             /* [rows,N] critic V(obs) or NULL */
  float* obs_copy;          /* [rows,N,12] or NULL */
  const float* last_start;  /* [N] episode_starts of this step or NULL */
  float* episode_starts;    /* [rows,N] or NULL */
  uint32_t* cursor;         /* device uint32[4] or NULL (t = 0, read-only without epilogue) */
  int32_t rows;             /* >= 1 */
  int32_t deterministic;    /* 1: a = mean (policy.predict(deterministic=True)) */
  uint64_t seed;
  uint64_t env_id_base;     /* global id of env 0 (keys the noise per env, shard-independent) */
  const QuadRolloutPost* epilogue;  /* fused epilogue of step t-1, or NULL */
} QuadPolicyAct;
int quad_policy_act(const float* packed, const QuadPolicyAct* a, int32_t n, void* stream);

/* Finish the pending step (end of a rollout): the epilogue for row (t-1) % rows if the cursor
 * marks one pending, then clears the mark. A no-op otherwise. */
int quad_rollout_post(const float* packed, const QuadRolloutPost* p, uint32_t* cursor, int32_t n,
                      void* stream);

/* ---- Fused rollout: `steps` whole steps of SB3 OnPolicyAlgorithm.collect_rollouts (train.py:50-68
 * drives it through SB3's PPO.learn) in ONE launch -- per step: policy (both MLPs on MFMA,
 * Gaussian sample, log-prob, clip), the env step of the handle (HoverEnv / TrajectoryFollowEnv,
 * optional RateControlWrapper, SB3 auto-reset), TimeLimit bootstrap, Monitor statistics, buffer
 * rows. Each 256-env block keeps its envs' state in registers and the packed weights in LDS for
 * all `steps`, so per step nothing is read from HBM. Results are bit-identical to the two-launch
 * form (quad_policy_act with epilogue + quad_step, then quad_rollout_post) with cursor t = t0.
 * Requires: a handle with env_kind HOVER or TRAJ, wrapper NONE or CTBR, auto_reset = 1.
 * Step t (t0 <= t < t0 + steps) writes row t % rows of the time-major buffers (every row pointer
 * required) and draws its action noise from Philox(seed; env_id_base + env, t, 0x200).
 * last_obs / last_start / ep_ret / ep_len carry the rollout across calls (read at entry, written
 * at exit); stats[slot] accumulate (finished return, length, count) as in QuadRolloutPost. */
typedef struct QuadRollout {
  float* obs_copy;          /* [rows,N,12] observation the step's action was taken from */
  float* actions;           /* [rows,N,4] unclipped sample (16-byte aligned) */
  float* log_prob;          /* [rows,N] */
  float* value;             /* [rows,N] V(obs) */
  float* episode_starts;    /* [rows,N] */
  float* rewards;           /* [rows,N] reward (+ gamma V(terminal_obs) on time-limit truncation) */
  float* last_obs;          /* [N,12] in: obs of step t0; out: obs after the last step */
  float* last_start;        /* [N] in/out: 1.0 where the next step begins an episode */
  float* ep_ret;            /* [N] in/out: running episode return */
  float* ep_len;            /* [N] in/out: running episode length */
  double* stats;            /* [QUAD_POLICY_STAT_SLOTS][3], accumulated */
  int32_t rows;             /* >= 1 */
  int32_t t0;               /* >= 0 */
  int32_t steps;            /* >= 1 */
  int32_t deterministic;    /* 1: a = mean */
  uint64_t seed;            /* action-noise seed */
  float gamma;
} QuadRollout;
int quad_rollout(QuadHandle* h, const float* packed, const QuadRollout* r, void* stream);

/* ---- PPO minibatch gradient on MFMA (row P): the gradient of SB3 PPO.train's minibatch loss
 * (stable_baselines3 ppo.py, as train.py:50-68 configures it; ppo/ppo.py ppo_loss restates it)
 *   loss = -mean(min(A r, A clip(r, 1 - clip_range, 1 + clip_range)))
 *          + ent_coef * (-entropy) + vf_coef * mean((returns - V)^2),
 *   r = exp(log_prob(actions) - old_log_prob), A = (adv - mean(adv)) / (std(adv) + 1e-8) over the
 *   minibatch (unbiased std; skipped when normalize_advantage == 0 or batch == 1),
 * with respect to every policy parameter, for the ActorCritic of QuadPolicyParams. Rows of the
 * flattened rollout buffer are gathered through `index` (a slice of the epoch's permutation), so
 * no minibatch copy is made. Ties of the min and the clip bounds follow torch's autograd
 * (torch.min splits a tie's gradient in half; clamp passes it on the closed interval). Gradients
 * are OVERWRITTEN (not accumulated) into `grads` (same shapes as the parameters); nothing in the
 * launch sequence synchronizes the host, so it is graph-capturable. */
typedef struct QuadPolicyGrads {
  float *pi_w0, *pi_b0, *pi_w1, *pi_b1, *act_w, *act_b;
  float *vf_w0, *vf_b0, *vf_w1, *vf_b1, *val_w, *val_b;
  float* log_std;
} QuadPolicyGrads;

typedef struct QuadPPOBatch {
  const float* obs;         /* [M,12] rollout buffer rows (16-byte aligned) */
  const float* actions;     /* [M,4] unclipped actions (16-byte aligned) */
  const float* log_prob;    /* [M] old log-probabilities */
  const float* advantages;  /* [M] */
  const float* returns;     /* [M] */
  const int64_t* index;     /* [batch] rows of this minibatch, each in [0, M) */
  int32_t batch;            /* >= 1 */
  int32_t normalize_advantage;  /* 0: off; 1: on; QUAD_ADV_PRECOMPUTED: on, and quad_ppo_adv_stats already
                                   wrote this minibatch's sums into the same workspace (stream-ordered);
                                   QUAD_ADV_GIVEN: on, with the sums in adv_sums */
  float clip_range, ent_coef, vf_coef;
  float* stats;             /* [4] out, or NULL: pg_loss, vf_loss, entropy, clip_fraction */
  const double* adv_sums;   /* QUAD_ADV_GIVEN: this minibatch's [QUAD_ADV_SUM_DOUBLES] block sums (a slice of
                               quad_ppo_adv_stats_epoch's output); ignored otherwise (ABI v5) */
} QuadPPOBatch;

/* ---- The optimizer step of PPO.train (row P), fused: torch.nn.utils.clip_grad_norm_(params,
 * max_grad_norm) followed by torch.optim.Adam.step() (SB3's policy optimizer, eps = 1e-5 in
 * train.py's policy_kwargs) over up to QUAD_ADAM_MAX_TENSORS device fp32 tensors, in two launches:
 *   total = ||all grads||_2; coef = min(max_grad_norm / (total + 1e-6), 1); grad *= coef
 *   (skipped when max_grad_norm <= 0); step += 1; m = b1 m + (1 - b1) g; v = b2 v + (1 - b2) g^2;
 *   p -= lr / (1 - b1^step) * m / (sqrt(v) / sqrt(1 - b2^step) + eps).
 * `step` points at each tensor's step counter (torch's float32 state["step"]); all are incremented. */
enum { QUAD_ADAM_MAX_TENSORS = 16 };
typedef struct QuadAdam {
  float* params[QUAD_ADAM_MAX_TENSORS];
  float* grads[QUAD_ADAM_MAX_TENSORS];       /* clipped in place, as clip_grad_norm_ does */
  float* exp_avg[QUAD_ADAM_MAX_TENSORS];
  float* exp_avg_sq[QUAD_ADAM_MAX_TENSORS];
  float* step[QUAD_ADAM_MAX_TENSORS];
  int32_t numel[QUAD_ADAM_MAX_TENSORS];
  int32_t count;                             /* tensors in use, 1..QUAD_ADAM_MAX_TENSORS */
  float max_grad_norm;
  double lr, beta1, beta2, eps;              /* moments and step size are formed in float64 */
} QuadAdam;
/* Device workspace (bytes) quad_clip_adam needs (gradient-norm partials). */
int64_t quad_adam_workspace_bytes(const QuadAdam* a);
int quad_clip_adam(const QuadAdam* a, void* workspace, int64_t workspace_bytes, void* stream);

/* The epoch permutation of PPO.train (SB3: np.random.permutation(buffer_size), the minibatch
 * index source of train.py:50-68's learner): out[i], i < n, is a permutation of [0, n) keyed by
 * `seed` -- a 4-round Feistel bijection of [0, 4^k) (4^k < 4n) restricted to [0, n) by cycle
 * walking. Device int64 [n]; n in [1, 2^40]. */
int quad_permutation(int64_t n, uint64_t seed, int64_t* out, void* stream);

/* Device workspace (bytes) quad_ppo_grad needs for a minibatch of `batch` rows. */
int64_t quad_ppo_workspace_bytes(int32_t batch);
/* Which kernel quad_ppo_grad launches: 1 = k_ppo_grad_x3 (bf16 MFMA on three-piece splits of every
 * f32 operand, f32-level error; the default), 0 = k_ppo_grad (f32-input MFMA; environment
 * QUADENV_LEARNER=f32, read on every call). Both meet the same accuracy bar. */
int quad_ppo_grad_form(void);
int quad_ppo_grad(const QuadPolicyParams* params, const QuadPPOBatch* b, const QuadPolicyGrads* grads,
                  void* workspace, int64_t workspace_bytes, void* stream);
/* The minibatch advantage statistics quad_ppo_grad's normalization needs (sum, sum of squares,
 * float64), on their own: a data-parallel learner enqueues them for the NEXT minibatch while the
 * gradient all-reduce of this one is in flight (they read only advantages[index]), then calls
 * quad_ppo_grad with normalize_advantage = QUAD_ADV_PRECOMPUTED and the same workspace. */
enum { QUAD_ADV_PRECOMPUTED = 2, QUAD_ADV_GIVEN = 3 };
int quad_ppo_adv_stats(const QuadPPOBatch* b, void* workspace, int64_t workspace_bytes, void* stream);
/* The same statistics for every minibatch of an epoch in ONE launch (SB3 PPO.train normalizes each
 * minibatch by its own mean / std; minibatch m is rows perm[m * batch .. (m + 1) * batch) of the
 * epoch permutation): sums[m * QUAD_ADV_SUM_DOUBLES ...] receives minibatch m's block sums in the
 * fixed order quad_ppo_adv_stats uses, so quad_ppo_grad with normalize_advantage = QUAD_ADV_GIVEN and
 * adv_sums = that slice gives bit-identical gradients. One full-occupancy launch per epoch instead
 * of n_minibatches latency-bound 256-block pre-passes. */
#define QUAD_ADV_SUM_DOUBLES 512
int quad_ppo_adv_stats_epoch(const float* advantages, const int64_t* perm, int32_t batch, int32_t n_minibatches,
                             double* sums, void* stream);
/* Diagnostics (parity tests): quad_ppo_grad through a build of the same kernel body that also
 * records the hidden pre-activations (before the ReLU) it computed for every minibatch row:
 * hidden[(net * batch + pos) * 256 + 128 * layer + neuron], net 0 = actor / 1 = critic, pos = the
 * row's position in `index`, layer 0 = h1 / 1 = h2 (device float32 [2][batch][256]). The gradients
 * are written as by quad_ppo_grad. Lets a test count the kernel's own ReLU decisions against
 * float64 (no reference interface: SB3 exposes no such hook). */
int quad_ppo_hidden(const QuadPolicyParams* params, const QuadPPOBatch* b, const QuadPolicyGrads* grads,
                    float* hidden, void* workspace, int64_t workspace_bytes, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* QUADENV_H */
