/* Host-side ABI exercise for the sanitizer build (tests/test_host_sanitize.py): every libffmp
 * entry point on the paths that need no GPU — argument and configuration validation, the
 * n == 0 no-op launches, the host footprint, layout / version / tuning queries, the DLPack
 * wrapper over host memory and its deleter, the ring pool query — run against a libffmp whose
 * host code is built with AddressSanitizer + UndefinedBehaviorSanitizer.  Exit 0 = every
 * expectation held (the sanitizers abort on their own findings). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ffmp.h"

static int failures = 0;
#define EXPECT(cond)                                                        \
  do {                                                                      \
    if (!(cond)) {                                                          \
      fprintf(stderr, "%s:%d: expectation failed: %s (last error: %s)\n", \
              __FILE__, __LINE__, #cond, ffmp_last_error());                \
      ++failures;                                                           \
    }                                                                       \
  } while (0)

/* dlpack.h (v0.8) layout, enough to reach the deleter */
typedef struct {
  void* data;
  int32_t device_type, device_id;
  int32_t ndim;
  uint8_t code, bits;
  uint16_t lanes;
  int64_t* shape;
  int64_t* strides;
  uint64_t byte_offset;
} dl_tensor_t;
typedef struct dl_managed {
  dl_tensor_t dl_tensor;
  void* manager_ctx;
  void (*deleter)(struct dl_managed*);
} dl_managed_t;

static void fill_cfg(ffmp_cfg_t* c, int grid, int n_obst, int n_beams) {
  memset(c, 0, sizeof(*c));
  c->grid = grid;
  c->n_obst = n_obst;
  c->n_beams = n_beams;
  c->max_steps = 200;
  c->moving = 1;
  c->autoreset = 1;
  c->collide_mode = FFMP_COLLIDE_FOOTPRINT | FFMP_COLLIDE_LIDAR;
  c->res = 0.05;
  c->dt = 0.1;
  c->robot_r = 0.13;
  c->goal_thr = 0.5;
  c->world_half = grid * 0.05;
  c->lidar_max = grid * 0.05 / 2;
  c->goal_min = 1.0;
  c->goal_max = grid * 0.05 / 2;
  c->obst_rmin = 0.1;
  c->obst_rmax = 0.3;
  c->obst_vmax = 0.5;
  c->start_clear = 0.5;
  c->goal_clear = 0.5;
  c->res_f = 0.05f;
  c->half_f = (float)(0.5 * grid * 0.05);
  c->world_half_f = (float)(grid * 0.05);
  c->half_ka_f = 0.5f;
  c->half_kr_f = 0.05f;
  c->rho0_f = 0.5f;
  c->inv_rho0_f = 2.0f;
  c->rho_min_f = 0.025f;
  c->inv_2res_f = 10.0f;
  c->cull_margin_f = 0.1f;
  c->seed = 7;
  c->n_foot = ffmp_footprint(grid, 0.05, 0.13, c->foot_di, c->foot_dj, FFMP_MAX_FOOT);
}

int main(void) {
  EXPECT(ffmp_abi_version() > 0);
  for (int k = 0; k <= 9; ++k) EXPECT(ffmp_layout(k) > 0);
  EXPECT(ffmp_layout(10) == -1 && ffmp_layout(-1) == -1);
  EXPECT(ffmp_layout(0) == (int64_t)sizeof(ffmp_cfg_t));

  /* host footprint: the reference's 21 cells at G = 64 / 100 / 256; the count is returned whatever
   * the capacity (at most `cap` written, NULL buffers = count only); bad grid / res refused */
  int32_t di[FFMP_MAX_FOOT], dj[FFMP_MAX_FOOT], d4[4], e4[4];
  EXPECT(ffmp_footprint(64, 0.05, 0.13, di, dj, FFMP_MAX_FOOT) == 21);
  EXPECT(ffmp_footprint(100, 0.05, 0.13, di, dj, FFMP_MAX_FOOT) == 21);
  EXPECT(ffmp_footprint(256, 0.05, 0.13, di, dj, FFMP_MAX_FOOT) == 21);
  EXPECT(ffmp_footprint(64, 0.05, 0.13, d4, e4, 4) == 21);
  EXPECT(d4[0] == di[0] && e4[3] == dj[3]);
  EXPECT(ffmp_footprint(64, 0.05, 0.13, NULL, NULL, 0) == 21);
  EXPECT(ffmp_footprint(0, 0.05, 0.13, di, dj, FFMP_MAX_FOOT) == FFMP_E_ARG);
  EXPECT(ffmp_footprint(64, -1.0, 0.13, di, dj, FFMP_MAX_FOOT) == FFMP_E_ARG);

  ffmp_cfg_t cfg;
  fill_cfg(&cfg, 64, 4, 0);
  EXPECT(cfg.n_foot == 21);
  ffmp_state_t st;
  ffmp_obs_t ob;
  ffmp_out_t out;
  memset(&st, 0, sizeof st);
  memset(&ob, 0, sizeof ob);
  memset(&out, 0, sizeof out);

  /* NULL buffers, bad configurations */
  EXPECT(ffmp_step(&cfg, 4, 0, NULL, &st, &ob, &out, NULL) == FFMP_E_ARG);
  EXPECT(strstr(ffmp_last_error(), "NULL") != NULL);
  EXPECT(ffmp_step(NULL, 4, 0, NULL, &st, &ob, &out, NULL) == FFMP_E_ARG);
  ffmp_cfg_t bad = cfg;
  bad.grid = 66;
  EXPECT(ffmp_raster(&bad, 1, NULL, NULL, &ob, NULL) == FFMP_E_CFG);
  bad = cfg;
  bad.n_obst = FFMP_MAX_OBST + 1;
  EXPECT(ffmp_raster(&bad, 1, NULL, NULL, &ob, NULL) == FFMP_E_CFG);
  bad = cfg;
  bad.n_foot = FFMP_MAX_FOOT + 1;
  EXPECT(ffmp_raster(&bad, 1, NULL, NULL, &ob, NULL) == FFMP_E_CFG);
  bad = cfg;
  bad.foot_di[0] = 1000;  /* footprint cell outside the grid */
  EXPECT(ffmp_raster(&bad, 1, NULL, NULL, &ob, NULL) == FFMP_E_CFG);
  bad = cfg;
  bad.rho_min_f = 0.0f;  /* outside the exact sqrt / reciprocal domain */
  EXPECT(ffmp_raster(&bad, 1, NULL, NULL, &ob, NULL) == FFMP_E_CFG);
  ffmp_cfg_t lid;
  fill_cfg(&lid, 64, 4, 8);  /* beam_cs NULL with n_beams > 0 */
  EXPECT(ffmp_reset(&lid, 1, 0, NULL, 1, &st, &ob, NULL) == FFMP_E_CFG);
  double table[40];
  lid.beam_cs = (const double*)(((uintptr_t)table + 15u) / 16u * 16u + 8u);  /* 8-B aligned only */
  EXPECT(ffmp_reset(&lid, 1, 0, NULL, 1, &st, &ob, NULL) == FFMP_E_CFG);
  EXPECT(strstr(ffmp_last_error(), "16-byte") != NULL);
  EXPECT(ffmp_scan_collision(-1, 4, NULL, 0.13, NULL, NULL, NULL) == FFMP_E_ARG);
  EXPECT(ffmp_scan_collision_f64(-1, 4, NULL, 0.13, NULL, NULL, NULL) == FFMP_E_ARG);

  /* n == 0 with valid pointers: success, no launch */
  double dbuf[16];
  memset(dbuf, 0, sizeof dbuf);
  void* p = dbuf;
  ffmp_state_t st2 = {(double*)p, (double*)p, (double*)p, (double*)p, (double*)p, (int32_t*)p, (int32_t*)p,
                      (float*)p, (uint32_t*)p, NULL, NULL};
  ffmp_obs_t ob2 = {(float*)p, (float*)p, (float*)p, (float*)p, (float*)p, (float*)p, (float*)p, NULL, 0, 0,
                    FFMP_OBS_F32, 0};
  ffmp_out_t out2 = {(float*)p, (uint8_t*)p, (uint8_t*)p, (uint8_t*)p, (uint8_t*)p};
  const int64_t act[1] = {0};
  EXPECT(ffmp_step_state(&cfg, 0, 0, act, &st2, &ob2, &out2, NULL) == FFMP_OK);
  EXPECT(ffmp_raster(&cfg, 0, (const float*)p, NULL, &ob2, NULL) == FFMP_OK);
  EXPECT(ffmp_step_fused(&cfg, 0, 0, act, &st2, &ob2, &out2, 0, NULL) == FFMP_OK);
  {
    /* the skewed step: the env step must write the other record buffer */
    float other[4];
    EXPECT(ffmp_step_skewed(&cfg, 0, 0, act, &st2, &ob2, &out2, other, 0, 0, NULL) == FFMP_OK);
    EXPECT(ffmp_step_skewed(&cfg, 4, 0, act, &st2, &ob2, &out2, (const float*)p, 0, 0, NULL) == FFMP_E_ARG);
  }
  ob2.format = 7;  /* unknown observation format */
  EXPECT(ffmp_raster(&cfg, 0, (const float*)p, NULL, &ob2, NULL) == FFMP_E_ARG);
  ob2.format = FFMP_OBS_U8F16;
  EXPECT(ffmp_raster(&cfg, 0, (const float*)p, NULL, &ob2, NULL) == FFMP_OK);

  /* episode bookkeeping validation */
  ffmp_episode_t ep;
  memset(&ep, 0, sizeof ep);
  EXPECT(ffmp_episode_init(4, NULL, 0, &ep, NULL) < 0);
  EXPECT(ffmp_episode_update(4, &out2, 65, 0, 0.8, 0, &ep, NULL) < 0);

  /* exact-math self-check: bad selector / range */
  EXPECT(ffmp_check_exact_math(2, 0, 1, NULL, NULL, NULL) < 0);

  /* launch tuning: bad key refused, a valid one set and restored */
  EXPECT(ffmp_set_tuning(99, 0) < 0);
  const int32_t prev = ffmp_set_tuning(FFMP_TUNE_RASTER_CPB, 8192);
  EXPECT(prev >= 0);
  EXPECT(ffmp_set_tuning(FFMP_TUNE_RASTER_CPB, 1000) < 0);  /* not a multiple of 1024 */
  EXPECT(ffmp_set_tuning(FFMP_TUNE_RASTER_CPB, prev) == 8192);

  /* DLPack over host memory (device_type 1 = kDLCPU) and its deleter; bad arguments */
  float host[2 * 3 * 4];
  const int64_t shape[3] = {2, 3, 4}, strides[3] = {12, 4, 1};
  dl_managed_t* mt = (dl_managed_t*)ffmp_dlpack(host, 1, 0, 3, shape, strides, 32, NULL);
  EXPECT(mt != NULL);
  if (mt) {
    EXPECT(mt->dl_tensor.data == host && mt->dl_tensor.ndim == 3 && mt->dl_tensor.bits == 32);
    EXPECT(mt->dl_tensor.shape[2] == 4 && mt->dl_tensor.strides[0] == 12);
    mt->deleter(mt);
  }
  EXPECT(ffmp_dlpack(host, 1, 0, 9, shape, strides, 32, NULL) == NULL);
  EXPECT(ffmp_dlpack(host, 1, 0, 3, shape, strides, 12, NULL) == NULL);
  EXPECT(ffmp_dlpack(NULL, 1, 0, 3, shape, strides, 32, NULL) == NULL);

  /* ring helper: argument checks before any device call, pool query */
  EXPECT(ffmp_ring_create(0, 1 << 20, 4, NULL, 0, NULL, NULL, NULL) == FFMP_E_ARG);
  ffmp_ring_t* ring = NULL;
  void* base = NULL;
  int64_t stride = 0;
  EXPECT(ffmp_ring_create(0, 0, 4, NULL, 0, &ring, &base, &stride) == FFMP_E_ARG);
  EXPECT(ffmp_ring_create(0, 1 << 20, 1, NULL, 0, &ring, &base, &stride) == FFMP_E_ARG);
  EXPECT(ffmp_ring_destroy(NULL) == FFMP_OK);
  double info[5];
  EXPECT(ffmp_ring_info(NULL, info, 5) == FFMP_E_ARG);
  EXPECT(ffmp_ring_pool_bytes(-1) == 0);

  if (failures) {
    fprintf(stderr, "%d expectation(s) failed\n", failures);
    return 1;
  }
  printf("abi_sanitize: all host-side checks passed\n");
  return 0;
}
