/* c_abi_consumer.c — a plain-C consumer of libffmp (include/ffmp.h): no Python, no torch.
 * Allocates every buffer with hipMalloc, fills the config by hand, resets and steps N envs with
 * the temporal stack kept in place (a frame window of W frames per env, FFMP_RASTER_NEWEST), and
 * checks size-independent invariants:
 *   - every state_m cell is 0 or 255,
 *   - the older frame equals the previous newest frame for envs that did not reset,
 *   - a reset env's two frames are identical,
 *   - the gradient equals the central difference of the potential plane at the robot cell,
 *   - ffmp_scan_collision on the lidar output finds no beam inside robot_r for envs still running.
 * Build (tests/test_c_abi_consumer.py): plain gcc against include/ + /opt/rocm/include,
 * linked with libffmp.so and libamdhip64.so.  Exit code 0 = all checks passed. */
#include <hip/hip_runtime_api.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ffmp.h"

#define HIPCHK(x)                                                              \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      fprintf(stderr, "HIP error %s at line %d\n", hipGetErrorString(e_), __LINE__); \
      return 2;                                                                \
    }                                                                          \
  } while (0)
#define FFCHK(x)                                                               \
  do {                                                                         \
    int r_ = (x);                                                              \
    if (r_ != 0) {                                                             \
      fprintf(stderr, "libffmp error %d: %s (line %d)\n", r_, ffmp_last_error(), __LINE__); \
      return 3;                                                                \
    }                                                                          \
  } while (0)

static void* dalloc(size_t bytes) {
  void* p = NULL;
  if (hipMalloc(&p, bytes) != hipSuccess) return NULL;
  hipMemset(p, 0, bytes);
  return p;
}

int main(void) {
  const int64_t N = 512;
  const int G = 128, K = 12, L = 90, STEPS = 25, W = 4;
  if (ffmp_abi_version() != FFMP_ABI_VERSION) {
    fprintf(stderr, "ABI mismatch\n");
    return 4;
  }
  ffmp_cfg_t cfg;
  memset(&cfg, 0, sizeof(cfg));
  cfg.grid = G; cfg.n_obst = K; cfg.n_beams = L; cfg.max_steps = 10; cfg.moving = 1; cfg.autoreset = 1;
  cfg.collide_mode = FFMP_COLLIDE_FOOTPRINT | FFMP_COLLIDE_LIDAR;
  cfg.n_foot = ffmp_footprint(G, 0.05, 0.13, cfg.foot_di, cfg.foot_dj, FFMP_MAX_FOOT);
  if (cfg.n_foot != 21) { fprintf(stderr, "footprint %d cells\n", cfg.n_foot); return 5; }
  cfg.res = 0.05; cfg.dt = 0.1; cfg.robot_r = 0.13; cfg.goal_thr = 0.5;
  cfg.world_half = 0.5 * G * 0.05 * 0.7;  /* a tight world: walls and discs are hit often */
  cfg.lidar_max = 0.5 * G * 0.05; cfg.goal_min = 1.0; cfg.goal_max = 2.0;
  cfg.obst_rmin = 0.1; cfg.obst_rmax = 0.5; cfg.obst_vmax = 1.0; cfg.start_clear = 0.5; cfg.goal_clear = 0.5;
  cfg.res_f = (float)cfg.res; cfg.half_f = (float)(0.5 * (G * cfg.res)); cfg.world_half_f = (float)cfg.world_half;
  cfg.half_ka_f = (float)(0.5 * 1.0); cfg.half_kr_f = (float)(0.5 * 0.1); cfg.rho0_f = (float)0.5;
  cfg.inv_rho0_f = (float)(1.0 / 0.5); cfg.rho_min_f = (float)(0.5 * cfg.res); cfg.inv_2res_f = (float)(1.0 / (2.0 * cfg.res));
  cfg.cull_margin_f = 0.1f; cfg.seed = 12345;
  /* beam table {cos, sin}(-pi + l*2pi/L), float64, on the device */
  double* beams_h = (double*)malloc(sizeof(double) * 2 * L);
  for (int l = 0; l < L; ++l) {
    const double th = -M_PI + l * (2.0 * M_PI / L);
    beams_h[2 * l] = cos(th);
    beams_h[2 * l + 1] = sin(th);
  }
  double* beams = (double*)dalloc(sizeof(double) * 2 * L);
  HIPCHK(hipMemcpy(beams, beams_h, sizeof(double) * 2 * L, hipMemcpyHostToDevice));
  cfg.beam_cs = beams;

  const size_t G2 = (size_t)G * G, rec = FFMP_REC_HDR + 12 * K;
  ffmp_state_t st = {(double*)dalloc(N * 3 * 8), (double*)dalloc(N * 2 * 8), (double*)dalloc(N * 8),
                     (double*)dalloc(N * K * 4 * 8), (double*)dalloc(N * K * 8), (int32_t*)dalloc(N * 4),
                     (int32_t*)dalloc(N * 4), (float*)dalloc(N * rec * 4), (uint32_t*)dalloc(4),
                     NULL, NULL /* no terminal record / obs */};
  /* slot-major frame ring (W, N, G, G): state_m[e] = (slot p, slot p+1) of env e */
  float* frames = (float*)dalloc((size_t)W * N * G2 * 4);
  ffmp_obs_t ob = {frames, (float*)dalloc(N * 2 * 4), (float*)dalloc(N * 2 * 4),
                   (float*)dalloc(N * 4), (float*)dalloc(N * G2 * 4), (float*)dalloc(N * 2 * 4),
                   (float*)dalloc(N * L * 4), NULL, (int64_t)G2, (int64_t)N * (int64_t)G2,
                   FFMP_OBS_F32, 0};
  ffmp_out_t out = {(float*)dalloc(N * 4), (uint8_t*)dalloc(N), (uint8_t*)dalloc(N), (uint8_t*)dalloc(N),
                    (uint8_t*)dalloc(N)};
  int64_t* act = (int64_t*)dalloc(N * 8);
  uint8_t* scol = (uint8_t*)dalloc(N);
  float* smin = (float*)dalloc(N * 4);
  if (!st.pose || !ob.state_m || !ob.potential || !act) { fprintf(stderr, "alloc failed\n"); return 2; }

  hipStream_t s;
  HIPCHK(hipStreamCreate(&s));
  int p = 0; /* frame slot of state_m[:, 0] */
  FFCHK(ffmp_reset(&cfg, N, 0, NULL, 1, &st, &ob, s));
  FFCHK(ffmp_raster_ex(&cfg, N, st.record, NULL, &ob, 0, 0, s));

  float* sm = (float*)malloc(N * 2 * G2 * 4);
  float* prev_new = (float*)malloc(N * G2 * 4);
  float* pot = (float*)malloc(N * G2 * 4);
  float* grad = (float*)malloc(N * 2 * 4);
  uint8_t *done = (uint8_t*)malloc(N), *col = (uint8_t*)malloc(N), *sc = (uint8_t*)malloc(N);
  float* mr = (float*)malloc(N * 4);
  int64_t* act_h = (int64_t*)malloc(N * 8);
  HIPCHK(hipStreamSynchronize(s));
  /* gather the [older, newest] pairs of all envs into sm (N, 2, G2): two strided plane copies */
#define COPY_PAIRS()                                                                                  \
  do {                                                                                              \
    HIPCHK(hipMemcpy2D(sm, 2 * G2 * 4, ob.state_m, G2 * 4, G2 * 4, N, hipMemcpyDeviceToHost));      \
    HIPCHK(hipMemcpy2D(sm + G2, 2 * G2 * 4, ob.state_m + (size_t)N * G2, G2 * 4, G2 * 4, N,         \
                       hipMemcpyDeviceToHost));                                                     \
  } while (0)
  COPY_PAIRS();
  for (int64_t e = 0; e < N; ++e) memcpy(prev_new + e * G2, sm + (e * 2 + 1) * G2, G2 * 4);

  uint64_t rng = 88172645463325252ull;
  long resets = 0, collisions = 0;
  const int c = G / 2;
  for (int t = 0; t < STEPS; ++t) {
    for (int64_t e = 0; e < N; ++e) {
      rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
      act_h[e] = (int64_t)(rng % FFMP_N_ACTIONS);
    }
    HIPCHK(hipMemcpyAsync(act, act_h, N * 8, hipMemcpyHostToDevice, s));
    FFCHK(ffmp_step_state(&cfg, N, 0, act, &st, &ob, &out, s));
    /* slide the pair one frame; the older slot already holds the previous newest frame, so
     * only the new one is written (and the older one of envs that reset) — until the window
     * wraps, when both frames are written at slot 0 */
    int32_t flags = FFMP_RASTER_NEWEST;
    if (++p > W - 2) { p = 0; flags = 0; }
    ob.state_m = frames + (size_t)p * N * G2;
    FFCHK(ffmp_raster_ex(&cfg, N, st.record, NULL, &ob, 0, flags, s));
    HIPCHK(hipStreamSynchronize(s));
    COPY_PAIRS();
    HIPCHK(hipMemcpy(pot, ob.potential, N * G2 * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(grad, ob.grad, N * 2 * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(done, out.done, N, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(col, out.collide, N, hipMemcpyDeviceToHost));
    for (int64_t e = 0; e < N; ++e) {
      const float* f0 = sm + (e * 2) * G2;
      const float* f1 = sm + (e * 2 + 1) * G2;
      for (size_t q = 0; q < 2 * G2; ++q) {
        const float v = f0[q];
        if (v != 0.0f && v != 255.0f) { fprintf(stderr, "bad cell value %f\n", v); return 10; }
      }
      if (done[e]) {
        ++resets;
        if (memcmp(f0, f1, G2 * 4) != 0) { fprintf(stderr, "reset env %ld frames differ\n", (long)e); return 11; }
      } else if (memcmp(f0, prev_new + e * G2, G2 * 4) != 0) {
        fprintf(stderr, "env %ld: older frame != previous newest frame at step %d\n", (long)e, t);
        return 12;
      }
      memcpy(prev_new + e * G2, f1, G2 * 4);
      const float* P = pot + e * G2;
      const float gx = (P[(c + 1) * G + c] - P[(c - 1) * G + c]) * cfg.inv_2res_f;
      const float gy = (P[c * G + c + 1] - P[c * G + c - 1]) * cfg.inv_2res_f;
      if (gx != grad[2 * e] || gy != grad[2 * e + 1]) { fprintf(stderr, "gradient mismatch env %ld\n", (long)e); return 13; }
      collisions += col[e];
    }
    /* is_collision2 on the float32 lidar output: an env that kept running has no beam inside
     * robot_r (the step applies the same predicate to the same float32 ranges) */
    FFCHK(ffmp_scan_collision(N, L, ob.lidar, cfg.robot_r, scol, smin, s));
    HIPCHK(hipStreamSynchronize(s));
    HIPCHK(hipMemcpy(sc, scol, N, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(mr, smin, N * 4, hipMemcpyDeviceToHost));
    for (int64_t e = 0; e < N; ++e) {
      if (!done[e] && sc[e]) {
        fprintf(stderr, "env %ld: lidar collision (%g m) but not done\n", (long)e, mr[e]);
        return 14;
      }
    }
  }
  uint32_t err = 0;
  HIPCHK(hipMemcpy(&err, st.err, 4, hipMemcpyDeviceToHost));
  printf("c_abi_consumer ok: N=%ld G=%d K=%d L=%d steps=%d resets=%ld collisions=%ld err=%u\n", (long)N, G, K, L,
         STEPS, resets, collisions, err);
  if (resets == 0 || collisions == 0 || err != 0) return 15;
  return 0;
}
