/*
 * ffmp.h — C ABI of libffmp, the MI355X (gfx950) batched flow-field
 * motion-planning environment (the `gym_ffmp` step/reset hot path).
 *
 * Every buffer is caller-owned, contiguous, env-major DEVICE memory (in
 * practice torch tensors' data_ptr()).  Nothing here allocates (except the
 * optional frame-ring helper ffmp_ring_create at the end), prints or throws.
 * Each call enqueues work on `stream` (a hipStream_t passed as void*;
 * NULL = the legacy default stream) and returns 0, or a negative FFMP_E_* code
 * with a message readable from ffmp_last_error() (thread-local).
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference repo YoshitakaNagai/flow_field_based_motion_planner):
 *   ffmp_reset          -> the external /episode_manager + is_first branch of
 *                          src/train.py:532-566 (start/goal, temporal stack
 *                          duplication, velocity := 0, d0 := dist) and the
 *                          commented-out FFMP.reset src/gym_ffmp/envs/ffmp.py:77-83
 *   ffmp_step, ffmp_step_fused -> one iteration of src/train.py:523-693 with Gazebo
 *                          (/cmd_vel integration), /bev_* rasterisers and
 *                          rewarder2 (src/gym_ffmp/envs/ffmp.py:179-188) in-GPU
 *   ffmp_ring_*, ffmp_dlpack -> storage of make_temporal_maps' 2-frame stack
 *                          (src/train.py:474-486) kept in place (optional helper)
 *   ffmp_temporal_maps  -> make_temporal_maps over INPUT_CHANNELS = k mono frames
 *                          (src/train.py:66-69, 474-486) served from the frame ring
 *   ffmp_bev_image      -> the (occupancy + flow(RGB)) image of the 12-channel option
 *                          (src/train.py:66, src/gym_ffmp/envs/ffmp.py:16)
 *   ffmp_raster         -> external /bev_flow_estimator + /temporal_bev_publisher
 *                          (src/train.py:116-121, make_temporal_maps :474-486)
 *   ffmp_reward_done    -> FFMP.rewarder / rewarder2 / reward_calculator /
 *                          is_goal / is_done (src/gym_ffmp/envs/ffmp.py:120-188)
 *   ffmp_footprint_collision -> FFMP.is_collision (ffmp.py:85-105)
 *   ffmp_scan_collision[_f64] -> FFMP.is_collision2 (ffmp.py:108-117)
 *   ffmp_footprint      -> the robot_grids mask built inside is_collision
 *                          (ffmp.py:87-94), host-side, float64
 *   ffmp_episode_init / ffmp_episode_update -> the main loop's episode
 *                          bookkeeping: counters src/train.py:501-505, reach_times /
 *                          reach_rate :579-587 (REACH_MEMORY_CAPACITY :76), is_first
 *                          :593,662, truncation :607, the is_done branch :611-682
 *                          (episode / step / total_step, completion test :644)
 */
#ifndef FFMP_H
#define FFMP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define FFMP_ABI_VERSION 8  /* 8: ffmp_step_skewed_check, ffmp_policy_reactive, ffmp_ring_va_reserved */
#define FFMP_MAX_OBST 64     /* K  */
#define FFMP_MAX_FOOT 128    /* footprint cells */
#define FFMP_MAX_BEAMS 1024  /* L  */
#define FFMP_N_ACTIONS 28
#define FFMP_REC_HDR 16      /* floats of per-env raster-record header */

/* error codes */
#define FFMP_OK 0
#define FFMP_E_ARG (-1)
#define FFMP_E_HIP (-2)
#define FFMP_E_CFG (-3)

/* collide_mode bits */
#define FFMP_COLLIDE_FOOTPRINT 1
#define FFMP_COLLIDE_LIDAR 2

/* Configuration, passed by pointer and copied by value into each launch.
 * float64 fields drive the per-env scalar maths (as the reference's Python
 * floats do); the *_f fields are the float32 constants of the per-cell raster
 * and MUST equal (float)(the double expression) documented beside them — the
 * Python host (flow_field_based_motion_planner_amd/config.py) fills both. */
typedef struct ffmp_cfg {
  int32_t grid;          /* G: local map is G x G cells, G % 4 == 0, 8 <= G <= 4096 */
  int32_t n_obst;        /* K: obstacles per env, 0..FFMP_MAX_OBST */
  int32_t n_beams;       /* L: lidar beams, 0..FFMP_MAX_BEAMS (0 = no lidar) */
  int32_t max_steps;     /* truncation: done when t == max_steps (train.py:60,607) */
  int32_t moving;        /* 1: obstacles move and reflect off the world walls */
  int32_t autoreset;     /* 1: ffmp_step resets done envs in place */
  int32_t collide_mode;  /* FFMP_COLLIDE_* bits */
  int32_t n_foot;        /* number of footprint offsets below */
  int32_t flow;          /* 1: raster the BEV motion-flow planes (obs.flow) */
  int32_t reserved0;
  int32_t foot_di[FFMP_MAX_FOOT]; /* footprint cell offsets from (G/2, G/2) */
  int32_t foot_dj[FFMP_MAX_FOOT];
  double res;            /* m per cell (ffmp.py:18, 0.05) */
  double dt;             /* s per step */
  double robot_r;        /* lidar collision threshold (ffmp.py:17, 0.13) */
  double goal_thr;       /* goal threshold (ffmp.py:19, 0.5) */
  double world_half;     /* world is [-world_half, world_half]^2 (m) */
  double lidar_max;      /* lidar max range (m); farther -> +inf */
  double goal_min, goal_max;   /* reset: goal distance range (m) */
  double obst_rmin, obst_rmax; /* reset: obstacle radius range (m) */
  double obst_vmax;            /* reset: obstacle speed range [0, vmax] (moving) */
  double start_clear, goal_clear; /* reset: clearance of obstacle surface from start / goal */
  /* float32 raster constants */
  float res_f;           /* (float)res */
  float half_f;          /* (float)(0.5 * (G * res)) : ego coordinate of cell 0 is -half_f */
  float world_half_f;    /* (float)world_half */
  float half_ka_f;       /* (float)(0.5 * k_att) */
  float half_kr_f;       /* (float)(0.5 * k_rep) */
  float rho0_f;          /* (float)rho0 : repulsive cut-off (m) */
  float inv_rho0_f;      /* (float)(1.0 / rho0) */
  float rho_min_f;       /* (float)rho_min : distance clamp (m) */
  float inv_2res_f;      /* (float)(1.0 / (2.0 * res)) : central-difference scale */
  float cull_margin_f;   /* extra culling margin (m), conservative */
  uint64_t seed;         /* Philox4x32-10 key */
  const double* beam_cs; /* DEVICE (L,2) float64 {cos, sin} of beam angle -pi + l*2pi/L, 16-B aligned */
} ffmp_cfg_t;

/* Per-env simulator state (device pointers, N envs). */
typedef struct ffmp_state {
  double* pose;     /* (N,3) x, y, yaw                               */
  double* goal;     /* (N,2) world goal                              */
  double* d0;       /* (N)   pre_relative_goal_dist (ffmp.py:139)    */
  double* obst;     /* (N,K,4) x, y, vx, vy                          */
  double* obst_r;   /* (N,K) radius                                  */
  int32_t* t;       /* (N)   steps since episode start               */
  int32_t* episode; /* (N)   episode counter (RNG key part)          */
  float* record;    /* (N, FFMP_REC_HDR + 12K) raster record */
  uint32_t* err;    /* (1)   sticky error bits (bit0: bad action id) */
  /* Optional (NULL = not written): the post-step state of every env BEFORE auto-reset, i.e. what
   * the reference loop observes on the iteration that ends an episode (train.py:543-557) —
   * consumers that store transitions (a replay memory) need it for done envs. Written by
   * ffmp_step / ffmp_step_state for all envs (equal to record / the small obs when not reset). */
  float* term_record; /* (N, FFMP_REC_HDR + 12K) */
  float* term_obs;    /* (N, 5) state_g[2], state_v[2], state_t */
} ffmp_state_t;

/* Observation plane formats (ffmp_obs_t.format).  F32: the reference consumer layout
 * (train.py:543-545 state_m float32 0/255; potential float32).  U8F16: a compact layout for
 * consumers that convert on load — state_m frames as uint8 0/255 (the same values) and the
 * potential plane as IEEE binary16 (float32 value rounded to nearest even); the state_m and
 * potential pointers then address uint8_t / binary16 elements and the state_m strides count
 * elements.  3 instead of 8 bytes per cell of a newest-only raster.  Flow planes (cfg.flow), when
 * present, are binary16 too (obs.flow then addresses binary16 elements). */
#define FFMP_OBS_F32 0
#define FFMP_OBS_U8F16 1

/* Observation tensors (device pointers).  Layout = reference train.py:44,543-557
 * with a leading N: state_m (N,2,G,G) [older, newest] values 0/255 as float. */
typedef struct ffmp_obs {
  float* state_m;   /* (N,2,G,G) */
  float* state_g;   /* (N,2) relative goal [dist, orient]          */
  float* state_v;   /* (N,2) per-step [|dxy|, wrap(dyaw)]          */
  float* state_t;   /* (N,1) dt (0 on the first step)              */
  float* potential; /* (N,G,G) attractive+repulsive potential, or NULL */
  float* grad;      /* (N,2) central-difference gradient at robot cell */
  float* lidar;     /* (N,L) ranges (+inf = no return, -inf = inside), NULL if L == 0 */
  float* flow;      /* (N,2,G,G) ego-frame velocity (m/s) of the disc covering each cell of the
                       newest frame (lowest disc index wins), 0 elsewhere; NULL unless cfg.flow */
  int64_t state_m_stride;       /* elements (floats) from env e's older frame to env e+1's; 0 = 2*G*G */
  int64_t state_m_frame_stride; /* floats from env e's older frame to its newest; 0 = G*G.
                                   0/0 is the contiguous (N,2,G,G) layout.  A slot-major frame
                                   window (W, N, G, G) uses G*G / N*G*G with state_m at the
                                   older slot (see FFMP_RASTER_NEWEST).  May be negative (the
                                   newest frame in a lower slot: a seamless ring's wrap step can
                                   write slot 0 through its first mapping instead of slot W's). */
  int32_t format;   /* FFMP_OBS_F32 (0) or FFMP_OBS_U8F16 */
  int32_t reserved;
} ffmp_obs_t;

/* Per-step outputs (device pointers, N each). Flags are 0/1 bytes. */
typedef struct ffmp_out {
  float* reward;
  uint8_t* done;
  uint8_t* is_goal;
  uint8_t* collide;
  uint8_t* truncated;
} ffmp_out_t;

int ffmp_abi_version(void);
const char* ffmp_last_error(void);

/* Layout check for FFI bindings: which = 0 sizeof(ffmp_cfg_t), 1 sizeof(ffmp_state_t),
 * 2 sizeof(ffmp_obs_t), 3 sizeof(ffmp_out_t), 4 offsetof(ffmp_cfg_t, res),
 * 5 offsetof(ffmp_cfg_t, res_f), 6 offsetof(ffmp_cfg_t, seed),
 * 7 offsetof(ffmp_cfg_t, beam_cs), 8 sizeof(ffmp_episode_t),
 * 9 offsetof(ffmp_obs_t, format); -1 otherwise. */
int64_t ffmp_layout(int32_t which);

/* Launch-shape tuning (process-wide; not thread-safe against concurrent launches).
 * Returns the previous value (>= 0) or FFMP_E_ARG.  Never changes results (FFMP_TUNE_CONV_MFMA: the
 * convolutions' fp32 summation order). */
#define FFMP_TUNE_RASTER_CPB 1  /* raster cells per block: multiple of 1024; 0 = default   */
#define FFMP_TUNE_RASTER_NT 2   /* raster stores: 0 by plane size, 1 plain, 2 nontemporal  */
#define FFMP_TUNE_RASTER_XCD 3  /* 1: XCD-aware block remap                                */
#define FFMP_TUNE_ENV_WAVES 4   /* waves per env_kernel block: 1 or 4                       */
#define FFMP_TUNE_ENV_LANES 5   /* lanes per env in env_kernel: 0 auto, 4, 8, 16, 32, 64 (a lane holds ceil(K / lanes) discs) */
#define FFMP_TUNE_RING_EXTRA 6  /* ffmp_ring_create / rebuild: fresh pieces allocated beyond the
                                   ones the ring needs (pairing candidates; they stay pooled):
                                   0 = default (need/2 + 4), v >= 1 = at most v - 1.  An HBM
                                   budget (FFMPVec hbm_budget) sets it around its ring creation. */
#define FFMP_TUNE_CONV_MFMA 7   /* MFMA shape of the convolution kernels that have both: 0 (default, each
                                   kernel's measured fastest: 32x32x16 for the forwards, the data gradient and
                                   the 32 -> 64 weight gradient, 16x16x32 for the other weight gradients and
                                   the small-image padded data gradients), 16
                                   (v_mfma_f32_16x16x32_bf16) or 32 (v_mfma_f32_32x32x16_bf16); the same
                                   products, fp32 sums in another order */
#define FFMP_TUNE_CONV_KYS 8    /* kernel rows per ring step of the row-ring convolution forward: 0 (default,
                                   1), 1, 2 or 4 (the same products and sums) */
#define FFMP_TUNE_CONV_LB 9     /* 1: the unpadded row-ring forward shares each tap's weights through LDS
                                   (one barrier per tap); 0 (default): from L1/L2 per wave */
#define FFMP_TUNE_CONV_WGPF 10  /* 1: the weight gradient reads each k-step's operands during the previous
                                   one's MFMAs (two register sets); 0 (default): not */
#define FFMP_TUNE_CONV_BA2 11   /* the 32 -> 64 unpadded row-ring forward (conv2) with each tap's loads pinned
                                   ahead of its MFMAs: 1 = B fragments two taps ahead (rows staged in 2
                                   registers), 2 = one tap ahead; 0 (default): the compiler's schedule */
#define FFMP_TUNE_CONV_MBW 12   /* 32-position blocks per wave of the row-ring forward: 0 (default) = by the
                                   grid-fill model (tiles of 512 / 384 / 256 / 128 positions), 1-4 forced */
#define FFMP_TUNE_CONV_PLANAR 13 /* 1: the row-ring forward keeps each 16-byte channel chunk of a row in a plane of
                                   its own (conflict-free A reads for any first column); 0 (default): padded cells */
#define FFMP_TUNE_CONV_PIN 14   /* 1: the row-ring forward's default launch with each half-trip's loads pinned ahead
                                   of its MFMAs by scheduling barriers; 0 (default): the compiler's schedule */
#define FFMP_TUNE_CONV_WGDMA 15 /* the weight gradient's stages copied by LDS-DMA into two LDS buffers (one barrier
                                   per stage): 0 (default) = with the k-step prefetch where the kernel runs one
                                   workgroup per CU (32 -> 64 channels), 1 = on, 2 = on with the prefetch, 3 = off,
                                   4 = the 32 -> 64 layer with 4 taps per wave, two workgroups per CU */
int32_t ffmp_set_tuning(int32_t key, int32_t value);

/* Host-side, float64: the footprint of ffmp.py:87-94 generalised to G
 * (map_range = G*res).  Writes up to `cap` offsets (cell - G/2); returns the
 * count, or a negative code. */
int ffmp_footprint(int32_t grid, double res, double robot_r,
                   int32_t* di, int32_t* dj, int32_t cap);

/* Reset envs [0,n) (global index env_offset + e) where mask[e] != 0 (mask NULL
 * = all).  initial != 0: episode := 0, else episode += 1.  Writes state, the
 * small obs (g, v=0, t=0, grad, lidar) and the raster record; call ffmp_raster
 * (same mask) afterwards for state_m / potential. */
int ffmp_reset(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset,
               const uint8_t* mask, int32_t initial,
               ffmp_state_t* state, ffmp_obs_t* obs, void* stream);

/* One env step for envs [0,n): action[e] in 0..27 (int64, train.py:343-345).
 * Integrates, moves obstacles, lidar, collision/goal/reward/done, truncation,
 * auto-reset (cfg.autoreset), small obs and raster record.  Does NOT raster. */
int ffmp_step_state(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset,
                    const int64_t* action, ffmp_state_t* state, ffmp_obs_t* obs,
                    ffmp_out_t* out, void* stream);

/* Raster state_m[:,0] (previous frame), state_m[:,1] (current frame) and the
 * potential plane from the raster record (mask NULL = all envs).  Record word 10 is 1 for a
 * record written by a reset (its two frames are identical), else 0. */
int ffmp_raster(const ffmp_cfg_t* cfg, int64_t n, const float* record,
                const uint8_t* mask, ffmp_obs_t* obs, void* stream);

/* ffmp_raster with an explicit launch shape (results are identical for every shape):
 * cells_per_block 0 (default 4096) or a multiple of 1024; flags FFMP_RASTER_*
 * (neither NT nor PLAIN: nontemporal stores for planes of <= 16K cells). */
#define FFMP_RASTER_NT 1     /* nontemporal 16-B stores          */
#define FFMP_RASTER_PLAIN 2  /* plain 16-B stores                */
#define FFMP_RASTER_XCD 4    /* XCD-aware block -> (env, tile) remap */
#define FFMP_RASTER_NEWEST 8 /* temporal stack in place (make_temporal_maps keeps the previous frame,
                                train.py:474-486): write state_m[:,1] (+ potential / flow) for every
                                env but state_m[:,0] only for envs whose record is a first frame
                                (reset: older == newest); the caller points state_m one frame past
                                the previous call's older slot, so [:,0] already holds the previous
                                newest frame */
#define FFMP_RASTER_TILE2 16 /* wave task = a 2 x 128-cell tile instead of 256 consecutive cells */
#define FFMP_RASTER_TILE4 32 /* 4 x 64-cell tile (compact cull box: fewer discs per task)       */
#define FFMP_RASTER_TILE8 64 /* 8 x 32-cell tile; any TILE flag needs G % (256/R) == 0 and blocks
                                of whole R-row bands (cells_per_block % (G*R) == 0 or >= G*G),
                                else the 256-cell chunks are used.  With FFMP_OBS_U8F16 and
                                G % 16 == 0 a wave task is 1024 cells (16 per lane): tiles are
                                R x 1024/R cells and need G % (1024/R) == 0 */
#define FFMP_RASTER_TILE16 256 /* 16 x 16-cell tile (compact 16 cells per lane: 16 x 64) */
#define FFMP_RASTER_NARROW 128 /* FFMP_OBS_U8F16: keep 4 cells per lane (256-cell wave tasks) */
#define FFMP_RASTER_MID8 512   /* FFMP_OBS_U8F16, G % 8 == 0: 8 cells per lane (512-cell wave tasks: an
                                  8-B frame and a 16-B potential store per lane; tiles R x 512/R);
                                  NARROW wins when both are set */
int ffmp_raster_ex(const ffmp_cfg_t* cfg, int64_t n, const float* record,
                   const uint8_t* mask, ffmp_obs_t* obs, int32_t cells_per_block,
                   int32_t flags, void* stream);

/* ffmp_step_state + ffmp_raster_ex in ONE launch (same results): one block per env, whose first
 * wave steps the env and whose 4 waves then raster its whole plane from the record just written
 * (flags as ffmp_raster_ex; cells_per_block is the whole plane, so TILE* needs only
 * G % (256/R) == 0).  The env step's float64 work overlaps other blocks' store streams instead
 * of running as its own launch. */
int ffmp_step_fused(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset, const int64_t* action,
                    ffmp_state_t* state, ffmp_obs_t* obs, ffmp_out_t* out, int32_t flags, void* stream);

/* The raster of step t and the env step of step t + 1 in ONE launch (round 5): the raster reads
 * record_raster (step t's record, written by the previous launch) and writes obs->state_m /
 * potential as ffmp_raster_ex does (cells_per_block, flags: the same meaning); the env step reads
 * action_next and advances state_next, whose record pointer must be the OTHER record buffer, and
 * writes the small obs (state_g/v/t, grad, lidar) and out of step t + 1.  Nothing either half reads
 * is written by the other, so the env waves' latency chains run beside raster blocks' stores.
 * Within a sequence of steps whose intermediate small outputs nobody reads (a replayed step graph:
 * ffmp_step_state of step 0 into buffer B, then this for t = 0 .. k-2 alternating the buffers, then
 * ffmp_raster_ex of step k-1) every frame, plane, state and record equals k ffmp_step calls.
 * Float32 frames without flow planes only (FFMP_E_ARG otherwise: run the two launches instead). */
int ffmp_step_skewed(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset, const int64_t* action_next,
                     ffmp_state_t* state_next, ffmp_obs_t* obs, ffmp_out_t* out, const float* record_raster,
                     int32_t cells_per_block, int32_t flags, void* stream);
/* Would ffmp_step_skewed take steps of this config in this obs format with these raster flags
 * (FFMP_RASTER_NT / PLAIN / XCD; NEWEST ignored)?  Runs every check of the launch — the env waves'
 * LDS (static arrays + 4 x envs-per-wave x L beam words) against the device's limit included — and
 * launches nothing.  FFMP_OK, or FFMP_E_ARG with the reason in ffmp_last_error().  A caller that
 * captures skewed step graphs asks this first (FFMPVec.capture) instead of re-deriving the LDS need. */
int ffmp_step_skewed_check(const ffmp_cfg_t* cfg, int32_t format, int32_t flags);

/* A scripted reactive controller — no reference counterpart (the reference's actions come from its
 * Q-network, src/train.py:336-347, published as /cmd_vel :665-682) — for closed-loop runs in which
 * step t + 1's action must be computed on the device from step t's observation (benchmarks, demos,
 * smoke tests).  Per env, from obs (the layout ffmp_step / ffmp_raster wrote: state_m's newest frame
 * through its strides and format, state_g):
 *   wi = clamp(rint(orient / 0.2) + 3, 0, 6)               (steer towards the goal)
 *   blocked = any newest-frame cell on the heading ray, rows G/2 + 3 .. G/2 + 3 + round(0.25 / res)
 *             of column G/2, is occupied (> 0)
 *   vi = blocked ? 0 : (dist < 1.0 m ? 1 : 3); blocked with wi == 3 -> wi = 6 (turn in place)
 *   action[e] = 7 * vi + wi   (RobotAction.cmd order, src/gym_ffmp/envs/robot/config.py:25-58)
 * action: (n) int64 device memory.  One thread per env, reads 8 + (look-ahead) cells' bytes. */
int ffmp_policy_reactive(const ffmp_cfg_t* cfg, int64_t n, const ffmp_obs_t* obs, int64_t* action, void* stream);

/* ffmp_step_state + ffmp_raster. */
int ffmp_step(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset,
              const int64_t* action, ffmp_state_t* state, ffmp_obs_t* obs,
              ffmp_out_t* out, void* stream);

/* Standalone reward/done (FFMP.rewarder / rewarder2 semantics), n envs:
 *   scan:   (n, scan_len) float64 ranges (0 = skipped, as `if scan_data[i]`), or NULL
 *   local_map: float32 planes, env e at local_map + e*map_stride (G x G), or NULL
 *   collide_in: optional precomputed collision bytes (used when scan and map are NULL)
 *   goal_in: optional precomputed goal bytes (NULL: dist < goal_thr)
 *   rel_goal (n,2) float64, is_first (n) bytes, d0 (n) float64 in/out.
 * Outputs reward (n) float64, done / is_goal / collide (n) bytes. */
int ffmp_reward_done(const ffmp_cfg_t* cfg, int64_t n,
                     const double* scan, int32_t scan_len,
                     const float* local_map, int64_t map_stride,
                     const uint8_t* collide_in, const uint8_t* goal_in,
                     const double* rel_goal, const uint8_t* is_first, double* d0,
                     double* reward, uint8_t* done, uint8_t* is_goal, uint8_t* collide,
                     void* stream);

/* One call of the single-env surface — FFMP.rewarder / rewarder2 / reward_calculator / is_goal
 * (src/gym_ffmp/envs/ffmp.py:120-188; rewarder2 is the one env call src/train.py:577 makes per
 * step) — from one packed buffer: host_buf (pinned host memory, 16-byte aligned) -> dev_buf (device,
 * >= in_bytes) in one copy, one ffmp_reward_done launch (n = 1), the 24 output bytes back into
 * host_buf in one copy, then the stream is synchronized: the results are in host_buf on return.
 * Layout (bytes): outputs reward f64 @0, d0 f64 @8 (in: the episode-start distance, out: set on
 * is_first), done / is_goal / collide u8 @16, 17, 18; inputs rel_goal f64[2] @24, is_first /
 * collide_in / goal_in u8 @40, 41, 42, scan f64[scan_len] @48, the local map f32[map_grid^2] @map_off
 * (16-aligned, >= 48 + 8 scan_len).  flags: 1 = collide_in given, 2 = goal_in given, 4 = a local map
 * (cfg's footprint; cfg->grid need not equal map_grid), 8 = without a map and with at most
 * FFMP_PACKED_ARG_BEAMS beams, pass the inputs as kernel arguments and write the outputs straight
 * into host_buf through its device view (hipHostGetDevicePointer: pinned, mapped memory) — one
 * launch and a synchronize, no copies; host_buf not mapped: the copies as without the flag. */
#define FFMP_PACKED_ARG_BEAMS 360
int ffmp_reward_done_packed(const ffmp_cfg_t* cfg, void* host_buf, void* dev_buf, int64_t in_bytes, int32_t scan_len,
                            int64_t map_off, int32_t map_grid, int32_t flags, void* stream);

/* FFMP.is_collision: any local_map[(G/2+di), (G/2+dj)] > 0 over the footprint. */
int ffmp_footprint_collision(const ffmp_cfg_t* cfg, int64_t n, const float* local_map,
                             int64_t map_stride, uint8_t* collide, void* stream);

/* FFMP.is_collision2 over (n, L) ranges: collide = any(r != 0 && r < thr);
 * min_r = min over those beams (+inf if none), may be NULL. */
int ffmp_scan_collision(int64_t n, int32_t L, const float* ranges, double thr,
                        uint8_t* collide, float* min_r, void* stream);
int ffmp_scan_collision_f64(int64_t n, int32_t L, const double* ranges, double thr,
                            uint8_t* collide, double* min_r, void* stream);

/* Self-check of the raster's exact fast math (no reference counterpart: the potential plane is
 * [no reference]): which = 0 compares sqrt_rn with sqrtf, 1 compares rcp_rn with
 * 1.0f / d, over the float bit patterns [lo_bits, hi_bits).  Adds the mismatch count to
 * *mismatches and atomic-mins the first mismatching pattern into *first_bits (device memory). */
int ffmp_check_exact_math(int32_t which, uint32_t lo_bits, uint32_t hi_bits,
                          unsigned long long* mismatches, uint32_t* first_bits, void* stream);

/* The learner's dominant convolution on the matrix cores (the reference
 * Network's conv2, src/train.py:233-242 / 244-255 — nn.Conv2d(32, 64, kernel_size=32) — and any
 * stride-1, unpadded convolution with 32 or 64 channels in and out):
 *   y[b][p][n] = act(bias[n] + sum_{ky,kx,c} x[b][yp+ky][xp+kx][c] * w[ky][kx][n][c])
 * x NHWC bf16 [batch][h][wd][c]; w bf16 [kh][kw][n][c] (torch's [n][c][kh][kw] permuted); bias
 * fp32 [n] or NULL; `pad` zero cells on every side of x (0 <= pad < kh, kw);
 * kernel column kx reads input column xo + kx * dx (dx >= 1: 1 = the plain convolution);
 * y NHWC [batch][h+2pad-kh+1][wd+2pad-(kw-1)dx][n], fp32 or (FFMP_CONV_OUT_BF16) bf16; fp32
 * accumulation on v_mfma_f32_32x32x16_bf16 (products exact, sums in fp32).  x and w 16-byte
 * aligned.  With pad = k - 1 and the kernel flipped and transposed (w'[ky][kx][c][n] =
 * w[k-1-ky][k-1-kx][n][c]) it is the data gradient of the unpadded convolution.
 * FFMP_CONV_W_FRAG: w holds the same elements in the kernels' fragment order,
 * [kh][kw][n/32][c/16][2][32][8] — weight (ky, kx, output channel o, input channel i) at index
 * ((((ky*kw + kx)*(n/32) + o/32)*(c/16) + i/16)*2 + (i%16)/8)*256 + (o%32)*8 + i%8 — so that each
 * 64-lane weight fragment load reads 1 KiB contiguous (the small-image kernel of conv3 / conv4:
 * ~17 % faster); the results are bit-identical to the plain layout's.
 * FFMP_CONV_X_FOLD (pad 0, dx = F >= 2 dividing c into an even count c / F): x is the UNFOLDED
 * NHWC input [batch][h][wd+F-1][c/F] of a few-channel convolution whose F consecutive kernel
 * columns were folded into channels; the kernel reads the folded image x'[b][y][x][j*(c/F) + i] =
 * x[b][y][x+j][i] — c / F <= 16 channels, wd columns — from it directly (no materialized fold).
 * Returns FFMP_OK or a negative code (ffmp_last_error()). */
#define FFMP_CONV_RELU 1
#define FFMP_CONV_OUT_BF16 2
#define FFMP_CONV_W_FRAG 4
#define FFMP_CONV_X_FOLD 8
int ffmp_conv2d_fwd_bf16(const void* x, const void* w, const float* bias, void* y, int32_t batch, int32_t h,
                         int32_t wd, int32_t c, int32_t kh, int32_t kw, int32_t n, int32_t pad, int32_t dx,
                         int32_t flags, void* stream);

/* The weight gradient of the same convolutions (MFMA, bf16 operands, fp32 accumulation):
 *   part[k][ky][kx][n][c] = sum over the samples of chunk k and all output positions p of
 *                           g[b][p][n] * x[b][yp+ky][xp+kx*dx][c]
 * g NHWC bf16 [batch][h-kh+1][wd-(kw-1)dx][n] (the output gradient), x NHWC bf16
 * [batch][h][wd][c] (the forward input); part fp32 [chunks][kh][kw][n][c] (every element
 * written); the caller sums over the chunks (batch split into `chunks` consecutive ranges). */
int ffmp_conv2d_wgrad_bf16(const void* g, const void* x, float* part, int32_t batch, int32_t h, int32_t wd, int32_t c,
                           int32_t kh, int32_t kw, int32_t n, int32_t dx, int32_t chunks, void* stream);

/* The data gradient of the same convolutions with the batch as the GEMM's M (the backward of
 * src/train.py:235's conv2 through autograd, :426-428):
 *   dx[b][Y][X][n] = sum_{ky,kx,c} g[b][Y+ky-(kh-1)][X+kx-(kw-1)][c] * w[ky][kx][c/8][n][c%8]
 * (cells outside g are zero: the full convolution).  g NHWC bf16 [batch][hy][wy][c] (the output
 * gradient); w bf16 [kh][kw][c/8][n][8] = the flipped, transposed kernel w'[ky][kx][n][c] =
 * w[n'=c][c'=n][kh-1-ky][kw-1-kx] with its channels in 8-blocks ahead of n; dx NHWC
 * [batch][hy+kh-1][wy+kw-1][n], fp32 or (FFMP_CONV_OUT_BF16) bf16.  32 samples share each MFMA
 * block, so every issued product is a useful one.  c = 32 or 64, n = 32; output rows of <= 72
 * positions; two gradient rows of KQ = 2 k-steps in LDS (wy <= 40). */
int ffmp_conv2d_dgrad_bf16(const void* g, const void* w, void* dx, int32_t batch, int32_t hy, int32_t wy, int32_t c,
                           int32_t kh, int32_t kw, int32_t n, int32_t flags, void* stream);

/* Would ffmp_conv2d_fwd_bf16 (kind 0; with pad > 0 the data-gradient form),
 * ffmp_conv2d_wgrad_bf16 (kind 1; pad ignored) or ffmp_conv2d_dgrad_bf16 (kind 2: h, wd = the
 * gradient's hy, wy; pad, dx ignored) accept this shape?  Runs every check of the launch
 * (channels, batch <= 65535, 16 KiB input rows, the LDS ring / stage, wgrad rows of >= 8
 * positions) and launches nothing.  FFMP_OK, or FFMP_E_ARG with the reason in ffmp_last_error().
 * The learner asks before it routes a convolution to the matrix-core kernels, and keeps the
 * library convolution for shapes outside them (src/train.py:231-303 at any map size). */
int ffmp_conv2d_check(int32_t kind, int32_t batch, int32_t h, int32_t wd, int32_t c, int32_t kh, int32_t kw,
                      int32_t n, int32_t pad, int32_t dx);

/* Episode bookkeeping of the training loop, batched (one record per env, device memory).
 * Per env and per ffmp_episode_update, exactly as src/train.py:579-682 does per iteration:
 *   reach window  <- is_goal (last `window` flags, window <= 64; REACH_MEMORY_CAPACITY = 10)
 *   reach_rate    =  np.average(window)                                    (:587, float64)
 *   done          =  out.done || (max_steps > 0 && step == max_steps)      (:607)
 *   done:  episode += 1, step = 0, is_first = 1, and with FFMP_EP_ARMED (the reference's
 *          `brain.loss != None`, :620) and reach_rate > threshold: complete = 1 (sticky, :644)
 *   else:  step += 1, total_step += 1, is_first = 0                       (:681-682)
 * FFMP_EP_RESET_ITER: the reference loop spends one iteration observing each freshly reset world
 * (is_first: never at the goal, never colliding) before an action takes effect; a batched env
 * folds it into the step that resets.  With this flag that iteration is run here as well — in
 * init and right after each done — so the counters equal the reference loop's.
 * Kept on purpose: the window counts iterations (not episodes), and the iteration that ends an
 * episode does not count towards total_step. */
#define FFMP_EP_TOTALS 8  /* totals[]: env-steps (updates), episodes, goals, collisions,
                             truncations, completions, counted steps (total_step increments), 0 */
#define FFMP_EP_ARMED 1
#define FFMP_EP_RESET_ITER 2
typedef struct ffmp_episode {
  uint64_t* reach_bits; /* (N) bit k = is_goal k iterations ago (bit 0 newest) */
  int32_t* reach_len;   /* (N) flags in the window (<= window) */
  double* reach_rate;   /* (N) */
  int32_t* step;        /* (N) iterations in the current episode */
  int32_t* episode;     /* (N) episodes ended */
  int64_t* total_step;  /* (N) */
  uint8_t* is_first;    /* (N) 1 before the first iteration of an episode */
  uint8_t* complete;    /* (N) sticky completion flag */
  uint64_t* totals;     /* (FFMP_EP_TOTALS) running sums over all envs, or NULL */
} ffmp_episode_t;

/* Start the masked envs (mask NULL: all, and totals zeroed) from the loop's initial values
 * (:501-505: counters 0, empty window, is_first = 1, complete = 0), followed by the
 * reset-observation iteration when flags has FFMP_EP_RESET_ITER. */
int ffmp_episode_init(int64_t n, const uint8_t* mask, int32_t flags, ffmp_episode_t* ep, void* stream);
/* One env step for envs [0,n) from its flags (out.done, out.is_goal, out.collide,
 * out.truncated; reward unused).  max_steps = 0 when out.done already includes truncation. */
int ffmp_episode_update(int64_t n, const ffmp_out_t* out, int32_t window, int32_t max_steps,
                        double threshold, int32_t flags, ffmp_episode_t* ep, void* stream);

/* make_temporal_maps (src/train.py:474-486) over k frames of the mono BEV image — the code path
 * of the reference's INPUT_CHANNELS = k with one image channel: map_memory keeps the last k
 * frames and is refilled with the first frame of an episode (is_first).  Served from a frame
 * window (the seamless ring keeps W >= k frames in place):
 *   out[e][c] = frame of lag d = k-1-c of env e (c = 0 oldest, k-1 newest), with the lag clamped
 *               to min(d, since[e]) — since = steps since the env's reset (ffmp_state_t.t), or
 *               NULL for no clamp;
 *   the frame of lag d of env e is at frames + lag_offset[d] + e * env_stride (elements;
 *   lag_offset a HOST array of k entries).
 * elem_bytes 1 (uint8 frames), 2 or 4 (float32); plane = G*G elements; out (n, k, G, G)
 * contiguous.  frames, out, plane * elem_bytes, env_stride * elem_bytes and every lag offset in
 * bytes must be 16-byte aligned.  A pure copy: k planes read and k written per env. */
#define FFMP_MAX_SERIES 16
int ffmp_temporal_maps(int64_t n, const void* frames, const int64_t* lag_offset, int32_t k, int64_t env_stride,
                       int64_t plane, int32_t elem_bytes, const int32_t* since, void* out, void* stream);

/* The 4-channel BEV image [occupancy, R, G, B] of the reference's 12-channel option
 * (src/train.py:66 "INPUT_CHANNELS = 12 #[channel] = (occupancy(MONO) + flow(RGB)) * series(3
 * steps)", src/gym_ffmp/envs/ffmp.py:16): the series of 3 such images is ffmp_temporal_maps over a
 * ring of them (plane = 4*G*G).  occ: the newest frame of env e at occ + e * occ_env_stride
 * (state_m's newest plane); flow: the (n, 2, plane) motion-flow planes of cfg.flow (ego vx, vy);
 * out: channel c of env e at out + e * out_env_stride + c * plane.  compact 0: float32 occ / flow /
 * out, compact 1 (FFMP_OBS_U8F16): uint8 occ and out, binary16 flow.  The reference's RGB flow
 * image came from BEV nodes outside its repository; the encoding here (float32, in this order):
 *   R = clamp(rint(127.5 + 127.5 * (vx / vmax)), 0, 255), G = the same of vy,
 *   B = clamp(rint(255 * (sqrt(vx*vx + vy*vy) / vmax)), 0, 255)   (rint: half to even)
 * — zero velocity is (128, 128, 0); vmax = the obstacle speed bound (FFMPConfig.obst_vmax). */
int ffmp_bev_image(int64_t n, int32_t compact, const void* occ, int64_t occ_env_stride, const void* flow,
                   int64_t plane, float vmax, void* out, int64_t out_env_stride, void* stream);

/* Seamless frame ring — an optional allocation helper (the step / raster entry points above
 * still never allocate).  The temporal stack of make_temporal_maps (src/train.py:474-486)
 * keeps the previous frame beside the new one; kept in place as a ring of `slots` frame
 * planes, the [older, newest] pair is the view of two consecutive slots [p, p+1].  A plain
 * array has no slot after the last one, so such a ring must wrap (and rewrite both frames)
 * every slots-1 steps.  This ring reserves (slots + 1) * slot_stride bytes of virtual address
 * space over `slots` physical slots of `device` (HIP virtual memory management) and maps
 * virtual slot `slots` onto the physical pages of slot 0 a second time, so the pair [p, p+1]
 * exists for every p in [0, slots): the view slides by one slot per step forever.
 *   Slots are built from physical pieces (1 GiB for slots of >= 2 GiB, else one per slot);
 *   slot_stride = slot_bytes rounded up to a whole number of pieces (out).
 *   partner (optional, device pointer, partner_bytes): the plane the raster writes in lockstep
 *   with every slot (the potential plane).  Two lockstep store streams run ~25 % slower when
 *   their physical pages pair badly, so each piece position gets a piece measured (two-stream
 *   store probe, which overwrites the partner's bytes) to pair well with the partner bytes the
 *   raster writes beside it: the same offset when partner_bytes < 1.5 x slot_bytes (float32
 *   frames beside a float32 plane), twice the offset otherwise (uint8 frames beside a binary16
 *   plane, FFMP_OBS_U8F16).  NULL: no pairing.  The library remembers the best probe per partner
 *   ADDRESS (the pairing reference, see ffmp_ring_pair_forget): a caller that passes a partner
 *   MUST call ffmp_ring_pair_forget(device, partner) when it frees that plane, or a plane
 *   allocated later at the same address inherits the old plane's reference (ffmp_ring_pool_trim
 *   does not forget them since ABI 8).
 *   *base = the first virtual slot (device pointer); contents undefined.
 * Returns 0, FFMP_E_ARG, or FFMP_E_HIP (no VMM support, out of memory, ...; then use a plain
 * ring — ffmp_last_error() says which call failed).
 * ffmp_ring_destroy drops the creator's reference.  Nothing is ever unmapped while the process
 * runs (ROCm 7 can resolve a reused, re-mapped VMM address to the old allocation — see
 * ffmp_kernels.hip): once a ring's last reference is gone its pieces return to a process-wide
 * pool that later rings draw from (or whose memory ffmp_ring_pool_trim gives back, keeping the
 * addresses reserved).  ffmp_ring_pool_bytes: pooled bytes (device < 0: all).
 * ffmp_ring_info: out[0..4] = pieces, fresh pieces allocated, pairing probes, min and max
 * probe GB/s of the chosen pieces (0 without a partner); with cap >= 6 also out[5] = the partner
 * byte ratio fixed at create (1: float32 frames beside a float32 plane, 2: uint8 frames beside a
 * binary16 plane; a rebuild keeps it).  Returns the number of values written (5 or 6). */
typedef struct ffmp_ring ffmp_ring_t;
int ffmp_ring_create(int32_t device, int64_t slot_bytes, int32_t slots, const void* partner,
                     int64_t partner_bytes, ffmp_ring_t** ring, void** base, int64_t* slot_stride);
/* A new ring (new addresses) with the pieces of `old`'s slots in replace_mask (bit i = slot i)
 * replaced by other pieces (chosen as in ffmp_ring_create, never the replaced ones), the other
 * slots' pieces shared with `old`.  For a caller whose timing shows a slot pairing badly.
 * `old` stays valid: the caller can time both rings and destroy the slower one (the kept
 * slots are the same memory in both, so only one of them should be written from then on).
 * A piece returns to the pool when the last ring holding it is gone; the pool is drawn from
 * only after a device synchronize (ffmp_ring_create / rebuild), so GPU work still writing a
 * dropped ring never overlaps the piece's next use. */
int ffmp_ring_rebuild(ffmp_ring_t* old, uint64_t replace_mask, const void* partner, int64_t partner_bytes,
                      ffmp_ring_t** ring, void** base, int64_t* slot_stride);
int ffmp_ring_destroy(ffmp_ring_t* ring);
int ffmp_ring_info(const ffmp_ring_t* ring, double* out, int32_t cap);
int64_t ffmp_ring_pool_bytes(int32_t device);
/* Bytes of virtual address space the ring helper has reserved on `device` in this process (piece
 * home mappings + every ring's (slots + 1) virtual slots).  Reservations are never freed while the
 * process lives (the re-map hazard above), so this only grows: a process that builds and drops rings
 * in a loop runs out of GPU virtual address space after roughly (device VA) / (per-ring delta)
 * rebuilds (INTEGRATION.md §5 states the bound measured for C3).  FFMP_E_ARG for device < 0 or >= 64. */
int64_t ffmp_ring_va_reserved(int32_t device);
/* Give back the physical memory of pooled pieces of `device` beyond the first keep_bytes
 * (0: all of them): after a device synchronize (pieces of rings dropped while kernels may still
 * write them are drained first), every mapping of such a piece — its home mapping and the slots
 * of the dead rings that held it — is unmapped and its handle released.  The address ranges
 * stay reserved until exit, so no later mapping is ever placed at an address that once held
 * another allocation (the stale-resolution hazard above).  Rings still alive are untouched, and
 * so are the pairing references (see ffmp_ring_pair_forget).  *released (optional) = bytes given
 * back.  Returns 0, FFMP_E_ARG or FFMP_E_HIP.  (FFMPVec calls it after construction and on close,
 * keeping FFMPVec.pool_keep_bytes: an instance's unchosen pairing candidates and the pieces of
 * rings it dropped go back to the device.)  Replaces no reference interface: the reference keeps
 * its 2-frame stack as a host NumPy array (src/train.py:474-486). */
int ffmp_ring_pool_trim(int32_t device, int64_t keep_bytes, int64_t* released);
/* The pairing references — the best two-stream probe seen per (device, partner plane), the
 * early-accept bar of ffmp_ring_create / ffmp_ring_rebuild — are keyed by the partner plane's
 * address.  The owner of a partner plane forgets its references when it frees the plane (a plane
 * allocated later at the same address must not inherit them): ffmp_ring_pair_forget(device,
 * partner), partner NULL = every reference of the device.  Returns the number forgotten (>= 0) or
 * FFMP_E_ARG.  ffmp_ring_pair_refs: how many the device holds. */
int ffmp_ring_pair_forget(int32_t device, const void* partner);
int ffmp_ring_pair_refs(int32_t device);
/* A dlpack.h (v0.8) DLManagedTensor* of `bits` elements (8: uint8, 16/32/64: float) over `data` (element strides,
 * ndim <= 8), for consumers that take DLPack (torch.utils.dlpack.from_dlpack, CuPy, JAX).
 * Its deleter frees it and, when `owner` is a ring, drops the reference it took on it: a ring
 * is parked once ffmp_ring_destroy was called AND every such tensor was deleted.
 * NULL on bad arguments. */
void* ffmp_dlpack(void* data, int32_t device_type, int32_t device_id, int32_t ndim, const int64_t* shape,
                  const int64_t* strides, int32_t bits, ffmp_ring_t* owner);

#ifdef __cplusplus
}
#endif
#endif /* FFMP_H */
