/*
 * voxnav.h -- C-ABI of the MI355X-native batched voxel-grid exploration env
 * (the hot path of Noimps/3D-Navigation-Reinforcement-Learning: envs/CubicEnv.py
 * step/reset, batched the way train/Grid_Train.py batches it through SB3's
 * SubprocVecEnv).  Implemented by libvoxnav.so (HIP, gfx950).
 *
 * Conventions
 *   - every function returns 0 on success and a negative VN_ERR_* code on
 *     failure; vn_last_error() returns a thread-local description.  No C++
 *     exception ever crosses this boundary.
 *   - "device" pointers are HIP device (HBM) pointers owned by the caller
 *     (e.g. torch tensors' data_ptr()), contiguous, naturally aligned.
 *   - `stream` is a hipStream_t passed as void* (NULL = default stream).
 *     All env calls are stream-ordered and asynchronous; none synchronises
 *     the host except to report a launch error.
 *   - one VnEnv per host thread; a VnEnv is bound to one device.
 *
 * Reference interfaces each entry point replaces are cited per function
 * (file:line into the reference tree).
 */
#ifndef VOXNAV_H
#define VOXNAV_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VN_ABI_VERSION 2
#define VN_OBS_DIM 80            /* envs/CubicEnv.py:58-62, :295-311 */
#define VN_VARIANT_CUBIC 0       /* envs/CubicEnv.py  (obs 80)                   */
#define VN_VARIANT_SIMPLE 1      /* envs/simpleEnv.py (obs 6L + 7, goal reward)   */
#define VN_MAX_OBS_DIM 103       /* 6 * VN_MAX_L + 7                              */
#define VN_STATE_FIELDS 16
#define VN_MAX_L 16              /* largest supported local_map_length */
#define VN_MAX_W 255
#define VN_MAX_D 255
#define VN_MAX_H 31
#define VN_MAX_ROOMS 256

enum {
    VN_OK = 0,
    VN_ERR_INVALID = -1,     /* bad argument (shape, range, NULL)          */
    VN_ERR_HIP = -2,         /* HIP runtime error                          */
    VN_ERR_ROOM = -3,        /* room has no interior free cell, too big... */
    VN_ERR_OOM = -4
};

typedef struct VnEnv VnEnv;

/*
 * Parsed rooms, exactly what GridAgent.load_room produces per room
 * (envs/CubicEnv.py:402-448): the dense grid with walls (grid == -2)
 * flagged, plus an optional "Start position".  Rooms are in the order the
 * caller wants random.choice to index (the build sorts file names).
 */
typedef struct VnRoomSet {
    int32_t n_rooms;
    const int32_t *whd;          /* [n_rooms][3]  W, D, H                       */
    const uint8_t *walls;        /* concat of W*D*H bytes, index (x*D+y)*H+z;
                                    CubicEnv: value -2 after its 2 -> -2 mapping
                                    (:434), simpleEnv: file value 2 (:282)      */
    const int32_t *fixed_start;  /* [n_rooms][3] or NULL; -1 = draw a start     */
    const int32_t *goal;         /* [n_rooms][3] or NULL; "Goal=" line, -1 =
                                    draw one (simpleEnv :419-426)               */
} VnRoomSet;

/* GridAgent ctor kwargs (envs/CubicEnv.py:17-29) + batching knobs. */
typedef struct VnConfig {
    int32_t local_map_length;    /* L (ctor default 4; Grid_Train uses 10)      */
    int32_t use_room_draw;       /* 1: room_path given -> random.choice(rooms)  */
    int32_t autoreset;           /* SB3 VecEnv auto-reset inside vn_step        */
    int32_t variant;             /* VN_VARIANT_CUBIC / VN_VARIANT_SIMPLE        */
    double crash_penalty;        /* ctor default -2.0                           */
    double finish_percentage;    /* FINISH_PERCENTAGE = 0.84 (CubicEnv.py:12)   */
    int64_t agent_id_base;       /* global id of this shard's agent 0           */
    int64_t seed_stride;         /* next episode seed = seed + stride (mod 2^32)*/
} VnConfig;

typedef struct VnInfo {
    int32_t n_agents;
    int32_t n_rooms;
    int32_t local_map_length;
    int32_t pad_w, pad_d, pad_h; /* belief map padding (max room dims, PH%4==0) */
    int64_t belief_bytes_per_agent;
    int64_t device_bytes;        /* total HBM owned by the env                  */
    int32_t variant;
    int32_t obs_dim;             /* floats per observation row                  */
} VnInfo;

const char *vn_last_error(void);
int vn_abi_version(void);

/* GridAgent.__init__ for N agents on `device` (envs/CubicEnv.py:17-74). */
int vn_create(const VnRoomSet *rooms, int32_t n_agents, const VnConfig *cfg, int32_t device, VnEnv **out);
int vn_destroy(VnEnv *env);
int vn_get_info(const VnEnv *env, VnInfo *info);

/*
 * GridAgent.reset(seed) for every agent with mask[i] != 0 (mask NULL = all)
 * (envs/CubicEnv.py:77-108, draws :407/:462).  seeds: device int64 [N],
 * each in [0, 2^32) (the reference also calls np.random.seed(seed), :80).
 * obs: device f32 [N][obs_dim]; rows of unmasked agents are left untouched.
 * simpleEnv variant (envs/simpleEnv.py:79-107): its reset neither seeds nor
 * returns an observation; the build seeds the draws with random.seed(seed)
 * and returns get_obs() after the reset (what train/evaluate_grid.py:54-55
 * does), so obs is that first observation.
 */
int vn_reset(VnEnv *env, const int64_t *seeds, const uint8_t *mask, float *obs, void *stream);

/*
 * GridAgent.step(action) for all N agents (envs/CubicEnv.py:110-132;
 * simpleEnv variant: envs/simpleEnv.py:109-150),
 * followed, when cfg.autoreset, by the SB3 VecEnv auto-reset of every agent
 * whose step ended the episode (terminated or truncated).
 *   actions       device i32 [N], each in 0..5
 *   obs           device f32 [N][obs_dim] (post-reset obs for finished agents;
 *                 obs_dim = 80, or 6L+7 for the simpleEnv variant)
 *   reward        device f32 [N]      (may be NULL)  -- f64 reward rounded
 *   reward64      device f64 [N]      (may be NULL)  -- exact f64 reward
 *   terminated    device u8  [N]      (may be NULL)
 *   truncated     device u8  [N]      (may be NULL)
 *   terminal_obs  device f32 [N][obs_dim] (may be NULL) written only for agents
 *                 that finished an episode in this step
 */
int vn_step(VnEnv *env, const int32_t *actions, float *obs, float *reward, double *reward64,
            uint8_t *terminated, uint8_t *truncated, float *terminal_obs, void *stream);

/*
 * k_steps fused steps under the build's uniform random policy
 * (action = (Philox4x32-10(key=policy_seed, ctr=(gid, t0+k))[0] * 6) >> 32).
 * Outputs are [k_steps][N]-major (obs [k_steps][N][80]); actions_out
 * (device i32 [k_steps][N]) may be NULL.
 */
int vn_step_random(VnEnv *env, uint64_t policy_seed, uint64_t t0, int32_t k_steps, int32_t *actions_out,
                   float *obs, float *reward, double *reward64, uint8_t *terminated, uint8_t *truncated,
                   float *terminal_obs, void *stream);

/*
 * Parity dumps.  state_out: device i64 [N][16] in the field order
 * x, y, z, facing, last_action, step_count, visited_count, bump_count,
 * done, last_bump, near_wall, was_near_wall, cells_insight_down, room,
 * max_steps, next_seed.  simpleEnv variant: fields 9..11 are the goal
 * (gx, gy, gz) and 12 is 0 (it has no last_bump / near-wall state).
 * belief_out: device i8 [N][pad_w][pad_d][pad_h] dense x-major, the
 * reference's internal_grid values (CubicEnv: -2 wall, -1 unknown, 0 free,
 * n visits; simpleEnv: -1 unknown, 0 free, 1 visited, 2 wall;
 * visit counts saturate at 63), cells outside the agent's room read -128.
 */
/*
 * Name of the kernel instantiation a call of this shape launches
 * (k_steps = 0: vn_reset; explicit_actions: vn_step; fast: reward, terminated
 * and truncated requested, no f64 reward or action record).  Diagnostics:
 * lets bench.py and rocprofv3 summaries name the kernel they time.  No
 * reference counterpart.
 */
int vn_kernel_label(const VnEnv *env, int32_t k_steps, int32_t explicit_actions, int32_t fast, char *buf,
                    int32_t len);
int vn_export_state(VnEnv *env, int64_t *state_out, void *stream);
int vn_export_belief(VnEnv *env, int8_t *belief_out, void *stream);

/*
 * GAE advantage/return scan (SB3 RolloutBuffer.compute_returns_and_advantage,
 * called from RecurrentPPO.learn at train/Grid_Train.py:228).  All arrays
 * device f32, [T][N]-major; last_values/dones [N].
 */
int vn_gae(const float *rewards, const float *values, const float *episode_starts, const float *last_values,
           const float *dones, int32_t T, int32_t N, double gamma, double gae_lambda, float *advantages,
           float *returns, void *stream);

/* ------------------------------------------------------------------------
 * Rollout collector (sb3_contrib RecurrentPPO.collect_rollouts, reached
 * from model.learn at train/Grid_Train.py:228; policy MlpLstmPolicy with
 * net_arch pi/vf=[256,256,128], lstm_hidden_size=256, :68-80, :196-204).
 * The GEMMs of the policy forward are library GEMMs issued by the caller;
 * these entry points are everything in between.  All device f32 unless
 * stated, stream-ordered.
 * ---------------------------------------------------------------------- */

/*
 * One LSTM step for n_lstm independent LSTMs over N agents (torch nn.LSTM
 * gate order i, f, g, o; RecurrentActorCriticPolicy._process_sequence):
 *   pre = gx + gh + b_ih + b_hh;  c = f*c + i*g;  h = o*tanh(c)
 *   gx       element (b, n, j) at gx[n*gx_row_stride + b*4H + j]  (x @ W_ih^T
 *            for all LSTMs in one GEMM)
 *   gh       [n_lstm][N][4H] (h @ W_hh^T) or NULL when the state is zero
 *   b_ih, b_hh [n_lstm][4H];  h (out), c (in/out) [n_lstm][N][H]
 *   h_store, c_store  [n_lstm][N][H] copies for the rollout buffer, or NULL
 * H must be a multiple of 4.
 */
int vn_lstm_cell(const float *gx, int64_t gx_row_stride, const float *gh, const float *b_ih, const float *b_hh,
                 float *h, float *c, float *h_store, float *c_store, int32_t n_lstm, int32_t N, int32_t H,
                 void *stream);

/*
 * vn_lstm_cell inside a rollout (RolloutCollector.collect, f32 policy): the
 * state is read from the buffer's lstm_c[t] (c_in, before the episode-start
 * mask) and the new (h, c) written only to lstm_h[t+1] / lstm_c[t+1]
 * (h_out, c_out); gh was computed from the unmasked lstm_h[t], so agents
 * with start[n] != 0 take neither gh nor c_in (their masked state is zero:
 * RecurrentActorCriticPolicy._process_sequence).  c_in != c_out; gh, start
 * non-NULL.  Other arguments as vn_lstm_cell.
 */
int vn_lstm_cell_masked(const float *gx, int64_t gx_row_stride, const float *gh, const float *b_ih,
                        const float *b_hh, const float *c_in, const float *start, float *h_out, float *c_out,
                        int32_t n_lstm, int32_t N, int32_t H, void *stream);

/* vn_lstm_cell with bf16 gate pre-activations (uint16_t storage) from bf16
 * GEMMs; the cell math and the (h, c) state stay f32, and h is also written
 * in bf16 to h_bf16 [n_lstm][N][H] (the next GEMMs' input), or NULL. */
int vn_lstm_cell_bf16(const uint16_t *gx, int64_t gx_row_stride, const uint16_t *gh, const float *b_ih,
                      const float *b_hh, float *h, float *c, uint16_t *h_bf16, float *h_store, float *c_store,
                      int32_t n_lstm, int32_t N, int32_t H, void *stream);

/*
 * The whole LSTM step of the bf16 policy path on the matrix cores: gate
 * GEMM [x | h] @ [W_ih | W_hh]^T (v_mfma_f32_32x32x16_bf16, f32 accumulate)
 * with the cell update as its epilogue.
 *   x        f32 [N][obs_dim] (the env's obs; rounded to bf16 in-kernel)
 *   h_in     bf16 [n_lstm][N][H] previous h (masked); h_out bf16, != h_in
 *   w_cat    bf16 [n_lstm][4H][Kp]: W_ih in columns [0, obs_dim), W_hh in
 *            [kx, kx+H), kx = obs_dim rounded up to 8, zeros elsewhere;
 *            Kp a multiple of 64 >= kx + H
 *   bias     f32 [n_lstm][4H] = b_ih + b_hh
 *   c        f32 [n_lstm][N][H] in/out; h32 / h_store / c_store f32 or NULL
 * H must be a multiple of 64.
 */
int vn_lstm_fused_bf16(const float *x, int32_t obs_dim, const uint16_t *h_in, const uint16_t *w_cat, int32_t Kp,
                       const float *bias, float *c, uint16_t *h_out, float *h32, float *h_store, float *c_store,
                       int32_t n_lstm, int32_t N, int32_t H, void *stream);

/*
 * vn_lstm_fused_bf16 inside a rollout (RolloutCollector.collect): the cell
 * state is read from the rollout buffer's previous slot and written only to
 * the next one, so no separate state array is rewritten every step.
 *   c_in   f32 [n_lstm][N][H]: the state entering the step BEFORE the
 *          episode-start mask (the buffer's lstm_c[t]); rows n with
 *          start[n] != 0 are read as zero (RecurrentActorCriticPolicy.
 *          _process_sequence's (1 - episode_start) mask); start f32 [N] or
 *          NULL (no mask)
 *   c_out  f32 [n_lstm][N][H], != c_in: the new state (lstm_c[t+1])
 *   h_store f32 or NULL: the new h (lstm_h[t+1])
 * Other arguments as vn_lstm_fused_bf16.
 */
int vn_lstm_fused_bf16_masked(const float *x, int32_t obs_dim, const uint16_t *h_in, const uint16_t *w_cat,
                              int32_t Kp, const float *bias, const float *c_in, const float *start, float *c_out,
                              uint16_t *h_out, float *h_store, int32_t n_lstm, int32_t N, int32_t H, void *stream);

/*
 * The whole LSTM step of the f32 (reference-dtype) policy path on the f32
 * matrix cores (v_mfma_f32_32x32x2_f32, exact f32 FMA chains): the gate GEMM
 * [x | h] @ [W_ih | W_hh]^T for n_lstm LSTMs with the cell update as its
 * epilogue, so the 4H gate pre-activations never reach memory
 * (RecurrentActorCriticPolicy._process_sequence for actor and critic,
 * sb3_contrib; replaces the two library GEMMs +
 * vn_lstm_cell_masked of one collector step).
 *   x        f32 [N][obs_dim], 16-byte aligned when obs_dim % 4 == 0
 *   h_in     f32 [n_lstm][N][H], != h_out; with start, rows n with
 *            start[n] != 0 are read as zero (the (1 - episode_start) mask)
 *   w_packed f32 [n_lstm][H/64][Kp][4][64]: element [b][ub][k][g][uu] =
 *            Wcat_b[g*H + 64*ub + uu][k], Wcat_b = [W_ih | 0 | W_hh] with
 *            W_ih in columns [0, obs_dim), W_hh in [kx, kx + H), kx =
 *            obs_dim rounded up to 16, Kp = kx + H
 *   bias     f32 [n_lstm][4H] = b_ih + b_hh
 *   c_in     f32 [n_lstm][N][H] (masked like h_in when start != NULL); may be
 *            c_out (in-place state)
 *   c_out, h_out  f32 [n_lstm][N][H]: the new state
 *   start    f32 [N] or NULL
 * H must be a multiple of 64.
 */
int vn_lstm_fused_f32(const float *x, int32_t obs_dim, const float *h_in, const float *w_packed, int32_t Kp,
                      const float *bias, const float *c_in, const float *start, float *c_out, float *h_out,
                      int32_t n_lstm, int32_t N, int32_t H, void *stream);

/*
 * One Linear layer (+ Tanh when tanh_act) of the policy's pi / vf MLPs
 * (MlpExtractor, net_arch [256, 256, 128] with Tanh, train/Grid_Train.py:68-80)
 * for n_branch (1 or 2) branches in one launch, on the f32 matrix cores with
 * the bias and Tanh in the epilogue:  y[i] = tanh(x[i] @ W_i^T + b_i).
 *   x[i]        f32 [M][K] rows with row stride ldx (>= K, % 4), 16-byte aligned
 *   w_packed[i] f32 [Nout/128][K][128]: element [cb][k][j] = W_i[128*cb + j][k]
 *   bias[i]     f32 [Nout];  y[i]  f32 [M][Nout]
 * K a multiple of 16, Nout a multiple of 128.  x, w_packed, bias and y are
 * host arrays of n_branch device pointers.
 */
int vn_linear_f32(int32_t n_branch, const float *const *x, int64_t ldx, const float *const *w_packed,
                  const float *const *bias, float *const *y, int32_t M, int32_t K, int32_t Nout, int32_t tanh_act,
                  void *stream);

/*
 * Action and value heads + Categorical draw (ActorCriticPolicy action_net /
 * value_net and distribution.get_actions / log_prob).
 *   latent_pi [N][P] (NULL: value only), latent_vf [N][P] (NULL: no value)
 *   w_action [n_actions][P], b_action [n_actions], w_value [P], b_value [1]
 *   actions (i32 [N]): Philox4x32-10(key=sample_seed, ctr=(agent_id_base+n,
 *   t | 2^63)) word 0 -> u = (w >> 8) / 2^24, first a with u < cdf[a]
 *   (argmax of the logits when deterministic); log_probs = logit - logsumexp.
 * n_actions <= 8, P a multiple of 4.
 */
int vn_policy_head(const float *latent_pi, const float *latent_vf, int32_t N, int32_t P, const float *w_action,
                   const float *b_action, int32_t n_actions, const float *w_value, const float *b_value,
                   uint64_t sample_seed, uint64_t t, int64_t agent_id_base, int32_t deterministic, int32_t *actions,
                   float *values, float *log_probs, void *stream);

/* vn_policy_head with bf16 latents (uint16_t storage); math in f32. */
int vn_policy_head_bf16(const uint16_t *latent_pi, const uint16_t *latent_vf, int32_t N, int32_t P,
                        const float *w_action, const float *b_action, int32_t n_actions, const float *w_value,
                        const float *b_value, uint64_t sample_seed, uint64_t t, int64_t agent_id_base,
                        int32_t deterministic, int32_t *actions, float *values, float *log_probs, void *stream);

/*
 * The collector's whole policy after the LSTM in ONE launch: the pi and vf
 * MLPs (MlpExtractor, Linear + Tanh per layer; net_arch [256, 256, 128],
 * train/Grid_Train.py:68-80) and the heads + Categorical draw of
 * vn_policy_head (ActorCriticPolicy.forward / predict_values), the
 * activations kept on chip (no latent reaches memory).  Replaces
 * vn_linear_f32 x n_layers + vn_policy_head of one collector step.
 *   n_branch 2: x[0] the pi input, x[1] the vf input; 1: x[0] the vf input
 *               (value only: the truncation bootstrap, last values)
 *   x[b]        f32 [M][K0] rows with row stride ldx (% 4), 16-byte aligned;
 *               K0 % 16 == 0, K0 <= 256
 *   widths      n_layers (1..4) layer widths, each 128 or 256; the last is P
 *   w_t[b * n_layers + l]  f32 W_l [N_l][K_l] packed per MFMA lane (16-byte
 *               aligned): [N_l/32][K_l/8][64][4], element [cb][kg][lane][s] =
 *               W_l[32 cb + lane % 32][8 kg + 4 (lane / 32) + s];
 *               K_0 = K0 rounded up to a multiple of 16 (zero weights past K0),
 *               K_l = widths[l - 1];  bias[b * n_layers + l] [N_l]
 *   w_action [n_actions][P], b_action (pi branch; n_actions <= 8),
 *   w_value [P], b_value [1]
 *   actions / log_probs (pi branch) and values: [M], the draw of
 *   vn_policy_head (Philox4x32-10 key sample_seed, counter (agent_id_base + m,
 *   t | 2^63); argmax when deterministic).
 * Host arrays: x (n_branch), widths (n_layers), w_t and bias (n_branch x n_layers).
 */
int vn_mlp_head_f32(int32_t n_branch, const float *const *x, int64_t ldx, int32_t K0, int32_t n_layers,
                    const int32_t *widths, const float *const *w_t, const float *const *bias, const float *w_action,
                    const float *b_action, int32_t n_actions, const float *w_value, const float *b_value,
                    uint64_t sample_seed, uint64_t t, int64_t agent_id_base, int32_t deterministic, int32_t *actions,
                    float *log_probs, float *values, int32_t M, void *stream);

/*
 * Ordered indices of the agents whose step was a time-limit truncation
 * (SB3 VecEnv: done and info["TimeLimit.truncated"] = truncated and not
 * terminated) -> boot_idx (device i32 [N]) and boot_count (device i32 [1]).
 * terminated / truncated must be 16-byte aligned.
 */
int vn_collect_compact(const uint8_t *terminated, const uint8_t *truncated, int32_t N, int32_t *boot_idx,
                       int32_t *boot_count, void *stream);

/*
 * Append the step's truncated agents (boot_idx / boot_count from
 * vn_collect_compact, device) to the rollout's bootstrap stash, so the
 * bootstrap values are computed once per rollout instead of after a host
 * read of the count every step (collect_rollouts' TimeLimit.truncated loop):
 * stash row base_in[0] + j takes agent a = boot_idx[j]'s terminal obs
 * (f32 [obs_dim]), its critic LSTM state (h_critic rows of H elements of
 * h_bytes = 2 (bf16) or 4 (f32) bytes, c_critic f32 rows; h_critic NULL: no
 * state) and the flat reward index t*N + a; base_out[0] = base_in[0] +
 * count (device i32).  Rows at or past cap are dropped: check the final
 * base <= cap.  Then vn_collect_bootstrap(stash_flat, values, M, gamma,
 * rewards [T][N]) applies them.
 */
int vn_collect_stash(const int32_t *boot_idx, const int32_t *boot_count, const int32_t *base_in, int32_t *base_out,
                     int32_t t, int32_t N, const float *terminal_obs, int32_t obs_dim, const void *h_critic,
                     int32_t h_bytes, const float *c_critic, int32_t H, float *stash_obs, void *stash_h,
                     float *stash_c, int32_t *stash_flat, int32_t cap, void *stream);

/*
 * Truncation bootstrap: rewards[boot_idx[i]] += gamma * terminal_values[i]
 * for i < M (f32, two roundings, as collect_rollouts' numpy update).
 */
int vn_collect_bootstrap(const int32_t *boot_idx, const float *terminal_values, int32_t M, double gamma,
                         float *rewards, void *stream);

/*
 * episode_starts[n] = terminated[n] | truncated[n] (f32 0/1, may be NULL)
 * and, for those agents, zero the LSTM state rows h, c [n_lstm][N][H] and
 * the bf16 copy h_bf16 (may be NULL) (n_lstm = 0: no recurrent state).
 */
int vn_episode_start(const uint8_t *terminated, const uint8_t *truncated, int32_t N, float *episode_starts,
                     float *h, float *c, uint16_t *h_bf16, int32_t n_lstm, int32_t H, void *stream);

/*
 * SB3 Monitor (train/Grid_Train.py:125 wraps every worker) for N agents, one
 * env step: ep_return (f64) += reward (reward64 when non-NULL, else the f32
 * reward), ep_length += 1; where terminated | truncated the finished
 * episode's (return, length) goes to rec_return / rec_length [N] (the
 * caller's row for this step; rec_length 0 = no episode ended) and the
 * counters restart, as Monitor.reset does under the VecEnv auto-reset.
 */
int vn_monitor_step(const double *reward64, const float *reward, const uint8_t *terminated, const uint8_t *truncated,
                    int32_t N, double *ep_return, int32_t *ep_length, double *rec_return, int32_t *rec_length,
                    void *stream);

/*
 * Everything the collector does after its env step t, in one launch:
 * episode_starts[n] = terminated | truncated (may be NULL); the Monitor step
 * (as vn_monitor_step, when ep_return is non-NULL; rec_* are the caller's
 * row t); the truncated (not terminated) agents' terminal obs and critic
 * state appended to the bootstrap stash (as vn_collect_compact +
 * vn_collect_stash, rows claimed atomically from *stash_count -- the
 * running count, read by the caller at a flush; rows past cap are dropped;
 * row order is not agent order, which the per-row bootstrap does not see);
 * and, for n_lstm > 0, the done agents' state rows h, c [n_lstm][N][H]
 * (and h_bf16, may be NULL) zeroed (as vn_episode_start).
 * Replaces sb3_contrib RecurrentPPO.collect_rollouts' per-step bookkeeping
 * after env.step (train/Grid_Train.py:228).
 */
int vn_collect_post_step(const uint8_t *terminated, const uint8_t *truncated, int32_t N, int32_t t,
                         float *episode_starts, const double *reward64, const float *reward, double *ep_return,
                         int32_t *ep_length, double *rec_return, int32_t *rec_length, const float *terminal_obs,
                         int32_t obs_dim, const void *h_critic, int32_t h_bytes, const float *c_critic, int32_t H,
                         float *stash_obs, void *stash_h, float *stash_c, int32_t *stash_flat, int32_t cap,
                         int32_t *stash_count, float *h, float *c, uint16_t *h_bf16, int32_t n_lstm, void *stream);

/* ------------------------------------------------------------------------
 * PPO learner: the LSTM re-run of sb3_contrib RecurrentPPO.train
 * (RecurrentActorCriticPolicy.evaluate_actions -> _process_sequence, from
 * model.learn at train/Grid_Train.py:228), its backward pass, and the
 * Linear layers of the update -- all on the library's own f32 matrix-core
 * kernels.  Gate order i, f, g, o (torch nn.LSTM).  All device f32,
 * stream-ordered.
 * ---------------------------------------------------------------------- */

/*
 * The learner's LSTM time loops on the f32 matrix cores (csrc/voxnav_learn_f32.hip;
 * sb3_contrib RecurrentPPO.train's LSTM re-run, train/Grid_Train.py:228, SURVEY.md
 * App. D.3): one launch per step, the whole product and the cell (or its backward)
 * fused.  vn_lstm_seq_pack_size gives the float counts of the two weight
 * workspaces (packed once per call).
 *   x      [L][B][D]                 w_ih [n_lstm][4H][D]   w_hh [n_lstm][4H][H]
 *   bias   [n_lstm][4H] = b_ih + b_hh
 *   hs, cs [n_lstm][L+1][B][H]       (index 0: the initial state, set by the caller)
 *   act    [L][n_lstm][B][4H]        (out: i, f, g, o after the nonlinearities)
 * Backward: dh_out [n_lstm][L][B][H] (gradient of the outputs), dG [n_lstm][L][B][4H]
 * (out), dc [n_lstm][B][H] (in: zeros = dL/dc_{L-1}; out: dL/dc_0), dh0 [n_lstm][B][H]
 * (out: dL/dh_0) or NULL.  D and H must be multiples of 4.
 */
int vn_lstm_seq_pack_size(int32_t n_lstm, int32_t D, int32_t H, int64_t *fwd_floats, int64_t *bwd_floats);
int vn_lstm_seq_fwd_mfma(const float *x, int32_t D, const float *w_ih, const float *w_hh, const float *bias,
                         float *wpack, float *hs, float *cs, float *act, int32_t n_lstm, int32_t L, int32_t B,
                         int32_t H, void *stream);
int vn_lstm_seq_bwd_mfma(const float *dh_out, const float *w_hh, float *wpack, const float *act, const float *cs,
                         float *dG, float *dc, float *dh0, int32_t n_lstm, int32_t L, int32_t B, int32_t H,
                         void *stream);

/*
 * The learner's LSTM re-run in the row layout (csrc/voxnav_learn_rows.hip; same
 * sb3_contrib RecurrentPPO.train re-run as above, train/Grid_Train.py:228): a
 * minibatch of R whole env rollouts as B = R rows over all L = T steps, a row's
 * state restarted from the buffer at every sequence start; ONE persistent launch
 * per direction with the weights resident in registers and the 8 unit blocks of
 * each (LSTM, 32-row tile) exchanging h (forward) / partial dh (backward) through
 * an in-launch agent-scope hand-off.  D 80, H 256, both LSTMs (actor, critic).
 *   x [L][B][D]; h_store, c_store [T][2][n_env][H] (the rollout buffer's states);
 *   env [L][B] int32 (the row's env), start [L][B] u8 (1: a sequence starts),
 *   keep [L][B] (1 - episode_start); out: hout, hprev (the h_{t-1} used), cprev,
 *   cnew [2][L][B][H], act [2][L][B][4H] (i, f, g, o); cnt: 2 * ceil(B / 32) * 64 u32 (one 256-B line per group counter)
 *   counters (zeroed by the call; 32-row tiles); err: set to 1 if a hand-off timed out.
 * Backward: dh_out [2][L][B][H] (+ the forward's hprev, cprev, cnew, act and x) ->
 * dG [2][L][B][4H] (may be NULL) and, accumulated inside the same launch, the weight gradients
 * dw_hh [2][4H][H], dw_ih [2][4H][D] and db_ih, db_hh [2][4H] (equal values, separate
 * storages: the parameters' own layouts); part:
 * vn_lstm_rows_part_floats floats of workspace.  vn_lstm_rows_supported: 1 when (D, H, B) can run (every
 * block co-resident on this device), else 0 (use vn_lstm_seq_*).
 */
int vn_lstm_rows_supported(int32_t D, int32_t H, int32_t B);
int vn_lstm_rows_part_floats(int32_t B, int64_t *floats);
int vn_lstm_rows_fwd(const float *x, int32_t D, const float *w_ih, const float *w_hh, const float *bias,
                     const float *h_store, const float *c_store, int64_t n_env, const int32_t *env,
                     const uint8_t *start, const float *keep, float *hout, float *hprev, float *cprev, float *cnew,
                     float *act, uint32_t *cnt, int32_t *err, int32_t L, int32_t B, int32_t H, void *stream);
int vn_lstm_rows_bwd(const float *dh_out, const float *w_hh, const float *act, const float *cprev, const float *cnew,
                     const float *hprev, const float *x, const uint8_t *start, float *dG, float *dw_hh,
                     float *dw_ih, float *db_ih, float *db_hh, float *part, uint32_t *cnt, int32_t *err, int32_t L,
                     int32_t B, int32_t H, void *stream);

/*
 * The learner's matrix products on the f32 matrix cores (csrc/voxnav_gemm_f32.hip):
 * every Linear of the PPO update (SB3 MlpExtractor / heads, RecurrentPPO.train) and
 * the LSTM weight gradients -- no library GEMM in the learner.  Batched over `batch`
 * with element strides s*.
 *   vn_gemm_f32_linear  C = act(A [M][K] @ W [N][K]^T + bias)   act 0 none, 1 tanh
 *   vn_gemm_f32_dx      C = dZ [M][K] @ W [K][N], dZ = dy (1 - y^2) (y != NULL) or dy
 *   vn_gemm_f32_tn      C [M][N] = dZ^T B, dZ [K][M] (as above), B [K][N], K split in
 *                       `splits` (workspace: splits*batch*M*N floats), colsum [batch][M]
 *                       = sum_k dZ[k][m] (workspace2: splits*batch*M), accumulate: C +=
 */
int vn_gemm_f32_linear(const float *a, int64_t lda, int64_t sa, const float *w, int64_t ldw, int64_t sw,
                       const float *bias, int64_t sbias, float *c, int64_t ldc, int64_t sc, int32_t M, int32_t N,
                       int32_t K, int32_t batch, int32_t act, void *stream);
int vn_gemm_f32_dx(const float *dy, const float *y, int64_t ldd, int64_t sd, const float *w, int64_t ldw, int64_t sw,
                   float *c, int64_t ldc, int64_t sc, int32_t M, int32_t N, int32_t K, int32_t batch, void *stream);
int vn_gemm_f32_tn(const float *dy, const float *y, int64_t ldd, int64_t sd, const float *b, int64_t ldb, int64_t sb,
                   float *c, int64_t sc, float *colsum, int32_t M, int32_t N, int32_t K, int32_t batch, int32_t splits,
                   float *workspace, float *workspace2, int32_t accumulate, void *stream);

/* PPO minibatch loss + its gradient to the MLP latents (csrc/voxnav_ppo_loss.hip).
 * Replaces, per minibatch, the heads and loss block of sb3 RecurrentPPO.train /
 * PPO.train (sb3_contrib ppo_recurrent.py train(): evaluate_actions -> ratio ->
 * clipped surrogate / value MSE / entropy -> loss.backward() down to the
 * latents), reached from train/Grid_Train.py:228 (model.learn).
 *   hp, hv [M][F] (row stride ldh): the actor / critic latents (F = 64..256, % 64)
 *   wa [A][F], ba [A] (action_net, A <= 8); wv [F], bv [1] (value_net)
 *   src [M] (NULL: identity): the buffer rows of the samples; actions int32,
 *   advantages, old_log_prob, returns: the rollout buffer, indexed by src
 *   -> dhp, dhv [M][F] contiguous: dloss/dlatent; grad_heads [A F + A + F + 1]:
 *      d action_net.weight, d action_net.bias, d value_net.weight, d value_net.bias;
 *      stats [6] f64: policy loss, value loss, entropy loss, loss, approx kl,
 *      clip fraction.  adv_sums [128] f64 scratch; part / spart: workspaces of
 *      the sizes vn_ppo_loss_part_floats returns (floats / doubles). */
int vn_ppo_loss_part_floats(int32_t M, int32_t F, int32_t A, int64_t *n_part, int64_t *n_spart);
int vn_ppo_loss(const float *hp, const float *hv, int64_t ldh, const float *wa, const float *ba, const float *wv,
                const float *bv, const int64_t *src, const int32_t *actions, const float *advantages,
                const float *old_log_prob, const float *returns, int32_t M, int32_t F, int32_t A, float clip_range,
                float ent_coef, float vf_coef, int32_t normalize_advantage, float *dhp, float *dhv, float *grad_heads,
                double *stats, double *adv_sums, float *part, double *spart, void *stream);

/* The total 2-norm of the parameter gradients (count <= 64 f32 tensors; device
 * pointers and element counts passed by host arrays) and the divisor the
 * fused Adam step applies to them: max(1, (norm + 1e-6) / max_norm), i.e.
 * 1 / torch.nn.utils.clip_grad_norm_'s clamped coefficient (sb3
 * max_grad_norm, sb3_contrib ppo_recurrent.py train()).  work: 256 doubles. */
int vn_grad_norm(const float *const *grads, const int64_t *sizes, int32_t count, float max_norm, float *norm,
                 float *scale, double *work, void *stream);

/* One Adam step over up to 64 f32 parameter tensors (torch.optim.Adam(eps,
 * betas), the optimizer sb3 builds for the policy; train/Grid_Train.py:84-86
 * lr 3e-4): the gradients divided by *clip_scale (vn_grad_norm's divisor; NULL:
 * 1), then torch's fused-Adam update with the bias corrections of `step`
 * (1-based); `steps` (nullable) receive the step count (torch's per-parameter
 * state["step"] scalars).  The gradients are not rewritten.  skip (nullable
 * device int32): when *skip != 0 at run time the launch changes nothing --
 * the learner passes the row-layout LSTM's error word (vn_lstm_rows_fwd/bwd
 * `err`), so gradients from a timed-out launch never reach the parameters. */
int vn_adam_step(float *const *params, const float *const *grads, float *const *exp_avg, float *const *exp_avg_sq,
                 float *const *steps, const int64_t *sizes, int32_t count, const float *clip_scale,
                 const int32_t *skip, float lr,
                 float beta1, float beta2, float eps, int64_t step, void *stream);

/* A PPO minibatch's rows (sb3 PPO.train over the env-major flattened rollout
 * buffer): sample i has env-major id idx[i] = env * T + t; src[i] receives its
 * row t * N + env of the [T, N]-major buffers and out[i] its observation
 * row (D floats, D % 4 == 0). */
int vn_minibatch_rows(const int64_t *idx, int32_t M, int32_t T, int32_t N, const float *obs, int32_t D, float *out,
                      int64_t *src, void *stream);

#ifdef __cplusplus
}
#endif
#endif /* VOXNAV_H */
