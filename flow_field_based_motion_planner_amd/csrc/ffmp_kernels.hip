// ffmp_kernels.hip — CDNA4 (gfx950) kernels + C ABI of libffmp.
//
// Kernels
//   env_kernel<MODE>   16/32/64 lanes per env (1-4 envs per wave): action -> unicycle integrate,
//                      obstacle motion, lidar (lane per beam), footprint
//                      collision (lane per footprint cell), goal/reward/done,
//                      truncation, auto-reset (Philox), gradient lookup, and the
//                      per-env raster record. Tiny per env; latency-hidden.
//   raster_kernel      the HBM-bound hot kernel: 256 threads x 4 cells per pass,
//                      writes the two float32 occupancy frames of state_m and
//                      the float32 potential plane with 16-B stores; obstacles
//                      staged in LDS and culled per 256-cell wave chunk.
//   step_raster_kernel the one-launch step: one block per env, env step then raster.
//   reward_done_kernel / footprint_kernel / scan_kernel — legacy FFMP methods.
// The seamless frame ring (HIP virtual memory) and the DLPack hand-off: ffmp_ring.hip.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <type_traits>
#include <cmath>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <stdarg.h>
#include <stddef.h>
#include <string.h>

#include "ffmp_device.h"

#pragma clang fp contract(off)

using namespace ffmp;

// The thread-local error message behind ffmp_last_error(), shared with ffmp_ring.hip.
namespace ffmp_detail {
thread_local char g_err[512] = "";

__attribute__((format(printf, 2, 3))) int fail(int code, const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
  return code;
}
int32_t ring_extra_swap(int32_t v);  // ffmp_ring.hip (FFMP_TUNE_RING_EXTRA)
int conv_mfma_swap(int v);           // ffmp_conv.hip (FFMP_TUNE_CONV_MFMA)
int conv_kys_swap(int v);            // ffmp_conv.hip (FFMP_TUNE_CONV_KYS)
int conv_lb_swap(int v);             // ffmp_conv.hip (FFMP_TUNE_CONV_LB)
int conv_wgpf_swap(int v);           // ffmp_conv.hip (FFMP_TUNE_CONV_WGPF)
int conv_ba2_swap(int v);            // ffmp_conv.hip (FFMP_TUNE_CONV_BA2)
int conv_mbw_swap(int v);            // ffmp_conv.hip (FFMP_TUNE_CONV_MBW)
int conv_planar_swap(int v);         // ffmp_conv.hip (FFMP_TUNE_CONV_PLANAR)
int conv_pin_swap(int v);            // ffmp_conv.hip (FFMP_TUNE_CONV_PIN)
int conv_wgdma_swap(int v);          // ffmp_conv.hip (FFMP_TUNE_CONV_WGDMA)
}  // namespace ffmp_detail
using ffmp_detail::fail;
using ffmp_detail::g_err;

namespace {

int check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    snprintf(g_err, sizeof(g_err), "%s: HIP launch failed: %s", what, hipGetErrorString(e));
    return FFMP_E_HIP;
  }
  return FFMP_OK;
}

int check_cfg(const ffmp_cfg_t* c) {
  if (!c) return fail(FFMP_E_ARG, "cfg is NULL");
  if (c->grid < 8 || c->grid > 4096 || (c->grid % 4) != 0)
    return fail(FFMP_E_CFG, "grid must be a multiple of 4 in [8,4096], got %d", c->grid);
  if (c->n_obst < 0 || c->n_obst > FFMP_MAX_OBST)
    return fail(FFMP_E_CFG, "n_obst out of range: %d", c->n_obst);
  if (c->n_beams < 0 || c->n_beams > FFMP_MAX_BEAMS)
    return fail(FFMP_E_CFG, "n_beams out of range: %d", c->n_beams);
  if (c->n_foot < 0 || c->n_foot > FFMP_MAX_FOOT)
    return fail(FFMP_E_CFG, "n_foot out of range: %d", c->n_foot);
  if (c->n_beams > 0 && !c->beam_cs) return fail(FFMP_E_CFG, "beam_cs is NULL with n_beams > 0");
  if (((uintptr_t)c->beam_cs & 15u) != 0) return fail(FFMP_E_CFG, "beam_cs must be 16-byte aligned");
  // the raster's sqrt_rn / rcp_rn are exact on this domain (ffmp_device.h)
  if (!(c->rho_min_f >= 0x1p-48f && c->rho_min_f <= 0x1p100f) || !(c->rho0_f <= 0x1p100f))
    return fail(FFMP_E_CFG, "rho_min must lie in [2^-48, 2^100] and rho0 <= 2^100");
  if (!(c->obst_rmin >= 0.0)) return fail(FFMP_E_CFG, "obst_rmin must be >= 0");
  for (int f = 0; f < c->n_foot; ++f) {
    const int i = c->grid / 2 + c->foot_di[f], j = c->grid / 2 + c->foot_dj[f];
    if (i < 0 || j < 0 || i >= c->grid || j >= c->grid)
      return fail(FFMP_E_CFG, "footprint cell outside the grid (index %d)", f);
  }
  return FFMP_OK;
}

int check_format(const ffmp_obs_t* o, bool flow) {
  if (o->format != FFMP_OBS_F32 && o->format != FFMP_OBS_U8F16)
    return fail(FFMP_E_ARG, "unknown obs.format %d", o->format);
  return FFMP_OK;
}

// Launch-shape tuning.  Defaults are the measured best on MI355X (profiles/r01_*);
// ffmp_set_tuning() (or the FFMP_RASTER_CPB / FFMP_RASTER_NT / FFMP_RASTER_XCD /
// FFMP_ENV_WAVES / FFMP_ENV_LANES environment variables, read once) overrides them for tuning
// sweeps.
struct Tuning {
  int cells_per_block = 4096;  // raster cells per block (multiple of 1024)
  int nontemporal = -1;        // raster store flavour: -1 by plane size, 0 plain, 1 nontemporal
  int xcd_remap = 0;           // 1: each XCD walks its own contiguous range of (env, tile) blocks
  int env_waves = 1;           // waves per env_kernel block: 1 or 4
  int env_lanes = 0;           // lanes per env: 0 = auto (>= K, more for many lidar beams)
  int lds_pad = 0;             // probe only (FFMP_RASTER_LDS_PAD): dynamic LDS bytes per raster block, to cap its occupancy
};

Tuning& tuning() {
  static Tuning t = [] {
    Tuning r;
    if (const char* v = getenv("FFMP_RASTER_CPB")) {
      const int c = atoi(v);
      if (c >= 1024 && c % 1024 == 0) r.cells_per_block = c;
    }
    if (const char* v = getenv("FFMP_RASTER_NT")) r.nontemporal = atoi(v) != 0 ? 1 : 0;
    if (const char* v = getenv("FFMP_RASTER_XCD")) r.xcd_remap = atoi(v) != 0 ? 1 : 0;
    if (const char* v = getenv("FFMP_ENV_WAVES")) r.env_waves = atoi(v) == 4 ? 4 : 1;
    if (const char* v = getenv("FFMP_RASTER_LDS_PAD")) r.lds_pad = std::max(0, std::min(atoi(v), 65536));
    if (const char* v = getenv("FFMP_ENV_LANES")) {
      const int l = atoi(v);
      r.env_lanes = (l == 4 || l == 8 || l == 16 || l == 32 || l == 64) ? l : 0;
    }
    return r;
  }();
  return t;
}

constexpr int kEnvMode_Step = 0;
constexpr int kEnvMode_Reset = 1;

__host__ __device__ inline int64_t rec_stride(int K) { return FFMP_REC_HDR + 12 * (int64_t)K; }

}  // namespace

// ============================================================================
// env_kernel: one wave (64 lanes) = one env; kEnvWaves envs per block.  Each wave only
// touches its own LDS slice, so waves synchronise with wave_sync() (no block barrier: waves
// of one block take different reset branches).
// ============================================================================

// Order LDS stores before other lanes' LDS loads within ONE wave (LDS ops of a wave complete
// in order; the fences stop the compiler from moving them across).
FFMP_DEV void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Probe builds only (-DFFMP_TRACE, tools/gpu_trace.sh; never the shipped libffmp): wall-clock
// stamps (100 MHz) at checkpoints of the env step (first 4096 envs, lane 0 of each env group)
// and of the raster (first 65536 blocks, thread 0), read back by ffmp_trace_read.  Each stamp
// first waits for the wave's outstanding memory operations, so the gaps are the chain's latency.
#ifdef FFMP_TRACE
__device__ uint64_t g_trace_env[4096 * 12];
__device__ uint64_t g_trace_ras[65536 * 4];
#define FFMP_ENV_STAMP(k)                                                   \
  do {                                                                      \
    __builtin_amdgcn_s_waitcnt(0);                                          \
    if (lane == 0 && e < 4096) g_trace_env[e * 12 + (k)] = wall_clock64();   \
  } while (0)
#define FFMP_RAS_STAMP(k)                                                                     \
  do {                                                                                        \
    __builtin_amdgcn_s_waitcnt(0);                                                            \
    if (threadIdx.x == 0 && blockIdx.x < 65536) g_trace_ras[blockIdx.x * 4 + (k)] = wall_clock64(); \
  } while (0)
#else
#define FFMP_ENV_STAMP(k) do {} while (0)
#define FFMP_RAS_STAMP(k) do {} while (0)
#endif

// One env's raster record: header, goal, then K float4 of each of cur / prev / vel.
// Lane k writes obstacle k; lanes 0..3 the header words.
FFMP_DEV void write_record_hdr(float* rec, int lane, const FrameHdr& hc, const FrameHdr& hp, float2 ge, float first) {
  if (lane == 0) {
    rec[8] = ge.x;
    rec[9] = ge.y;
    rec[10] = first;  // 1: written by a reset, the two frames are identical
    rec[11] = 0.0f;
  }
  if (lane < 4) {
    rec[lane] = lane == 0 ? hc.px : lane == 1 ? hc.py : lane == 2 ? hc.c : hc.s;
    rec[4 + lane] = lane == 0 ? hp.px : lane == 1 ? hp.py : lane == 2 ? hp.c : hp.s;
    rec[12 + lane] = 0.0f;
  }
}
// disc k of K: its current and previous ego disc and its ego velocity
FFMP_DEV void write_record_obst(float* rec, int k, int K, float4 ecur, float4 eprev, float4 vel) {
  float4* ro = reinterpret_cast<float4*>(rec + FFMP_REC_HDR);
  ro[k] = ecur;
  ro[K + k] = eprev;
  ro[2 * K + k] = vel;
}

// The lidar beam table {cos, sin} (cfg.beam_cs, (L, 2) float64) is read one beam ahead: lane
// `lane` of a group serves beams lane, lane + LPE, ...; the load of the next beam is in flight
// while the current one is traced, instead of a dependent round trip per beam.  first_beam is
// issued at the top of the env step, so the first load overlaps the integrator.
FFMP_DEV double2 first_beam(const ffmp_cfg_t& cfg, int lane) {
  return lane < cfg.n_beams ? reinterpret_cast<const double2*>(cfg.beam_cs)[lane] : make_double2(0.0, 0.0);
}

// Beams traced per lane at a time (trace_beams in ffmp_device.h); 1 = one beam at a time,
// lidar_beam with the table read one beam ahead.  3: C3's env kernel 87.4-88.3 -> 78.5-79.4 us, C5
// share 92.1 -> 82.8 (2 -> 80.7-81.3 / 85.2; 4 -> 92 at 131 VGPRs, 3 waves per SIMD;
// profiles/r03c_beam_chunk.txt), bit-identical ranges.
#ifndef FFMP_BEAM_CHUNK
#define FFMP_BEAM_CHUNK 3
#endif

template <class F>
FFMP_DEV void for_beams(const ffmp_cfg_t& cfg, int lane, int lpe, double2 b, F&& f) {
  const double2* bt = reinterpret_cast<const double2*>(cfg.beam_cs);
  for (int l = lane; l < cfg.n_beams; l += lpe) {
    const int ln = l + lpe;
    const double2 nb = ln < cfg.n_beams ? bt[ln] : make_double2(0.0, 0.0);
    f(l, b);
    b = nb;
  }
}

// The footprint offsets (cfg.foot_di / foot_dj) into the wave's LDS table, by every lane of the
// wave before any lane leaves (call ahead of the kernel's early returns; env_group's wave_sync
// orders it before the footprint test).  The kernel-argument segment is read uncached (~0.4 us a
// load, measured): read in the footprint loop itself, one dependent round trip per offset made the
// footprint 16 us of a C2 env step (profiles/r02_env_chain.txt); staged here, the loads of a wave
// overlap each other and the state loads.
// The footprint cells' ego coordinates do not depend on the env (the robot is cell (G/2, G/2) of
// every ego map), so they are staged as floats: cell_coord of each offset, the same float32
// operations the test made per env and cell (round 4).
// s_foot[FFMP_MAX_FOOT] gets the cells' extent {max |ex|, max |ey|} (a wave max; every lane of the
// wave must call this), which lets env_group skip the footprint test where it cannot fire.
FFMP_DEV void stage_footprint(const ffmp_cfg_t& cfg, float2* s_foot) {
  const int ic = cfg.grid / 2;
  float bx = 0.0f, by = 0.0f;
  for (int f = (int)(threadIdx.x & 63); f < cfg.n_foot; f += 64) {
    const float2 c = make_float2(cell_coord(cfg, ic + cfg.foot_di[f]), cell_coord(cfg, ic + cfg.foot_dj[f]));
    s_foot[f] = c;
    bx = fmaxf(bx, fabsf(c.x));
    by = fmaxf(by, fabsf(c.y));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    bx = fmaxf(bx, __shfl_xor(bx, o, 64));
    by = fmaxf(by, __shfl_xor(by, o, 64));
  }
  if ((threadIdx.x & 63) == 0) s_foot[FFMP_MAX_FOOT] = make_float2(bx, by);
}

// LPE lanes per env (16, 32 or 64 >= K): a wave serves 64 / LPE envs, so the per-env scalar
// float64 work (integrator, trig, goal, reward, record header) is issued once per 64/LPE envs
// instead of once per env; lane k of an env's group holds its obstacle k, beams and footprint
// cells are strided over the group's lanes.
// One env's step (or reset) by its LPE-lane group: lane = the lane within the group, s_* = the
// group's LDS slices (FFMP_MAX_OBST entries each).  Used by env_kernel and step_raster_kernel.
template <int MODE, int LPE, int BCH = FFMP_BEAM_CHUNK, bool DL = false, int DPL = 1>
FFMP_DEV __attribute__((always_inline)) void env_group(const ffmp_cfg_t& cfg, int64_t env_offset,
                                                       const int64_t* __restrict__ action, int32_t initial,
                                                       const ffmp_state_t& st, const ffmp_obs_t& ob,
                                                       const ffmp_out_t& out, int64_t e, int lane, double* s_ox,
                                                       double* s_oy, double* s_or, double* s_orr, float4* s_ecur,
                                                       float4* s_eprev, const float2* s_foot, float* s_rhdr = nullptr,
                                                       float2* s_rvel = nullptr, uint32_t* s_key = nullptr,
                                                       int* s_pref = nullptr, int* s_lo = nullptr) {
  static_assert(LPE == 4 || LPE == 8 || LPE == 16 || LPE == 32 || LPE == 64, "lanes per env");
  static_assert(DPL == 1 || DPL == 2 || DPL == 4, "discs per lane");
  const int K = cfg.n_obst;
  const int L = cfg.n_beams;
  const int G = cfg.grid;
  const int ic = G / 2;
  const int64_t genv = env_offset + e;
  FFMP_ENV_STAMP(0);
  const double2 beam0 = first_beam(cfg, lane);  // in flight during the integrator's chain

  // ---- load (uniform scalars in every lane; discs k = lane + j LPE, j < DPL, in this lane) ----
  double x0 = st.pose[e * 3 + 0], y0 = st.pose[e * 3 + 1], yaw0 = st.pose[e * 3 + 2];
  double gx = st.goal[e * 2 + 0], gy = st.goal[e * 2 + 1];
  double d0 = st.d0[e];
  int32_t t = st.t[e];
  int32_t episode = st.episode[e];
  Obst my[DPL];
  bool has_obst[DPL];
#pragma unroll
  for (int j = 0; j < DPL; ++j) {
    const int k = lane + j * LPE;
    has_obst[j] = k < K;
    my[j] = Obst{0.0, 0.0, 0.0, 0.0, 0.0};
    if (MODE == kEnvMode_Step && has_obst[j]) {
      const double* p = st.obst + (e * K + k) * 4;
      my[j].x = p[0]; my[j].y = p[1]; my[j].vx = p[2]; my[j].vy = p[3];
      my[j].r = st.obst_r[e * K + k];
    }
  }

  double x1 = x0, y1 = y0, yaw1 = yaw0;
  double c0 = 0.0, s0 = 0.0;
  double vlin = 0.0, vang = 0.0;
  float t_obs = 0.0f;
  bool reset_now = (MODE == kEnvMode_Reset);

  if (MODE == kEnvMode_Step) {
    // ---- action -> (v, w) (train.py:668-673 -> Gazebo /cmd_vel) ----
    int64_t a = action[e];
    if (a < 0 || a >= FFMP_N_ACTIONS) {
      if (lane == 0) atomicOr(st.err, 1u);
      a = 3;  // (0.0, 0.0)
    }
    const double v = cmd_v((int)a / 7), w = cmd_w((int)a % 7);
    // ---- unicycle integrator (SPEC a15) ----
    c0 = cos(yaw0);
    s0 = sin(yaw0);
    x1 = x0 + (v * c0) * cfg.dt;
    y1 = y0 + (v * s0) * cfg.dt;
    yaw1 = pi_to_pi(yaw0 + w * cfg.dt);
    // previous frame record from the pre-step pose / obstacle positions
#pragma unroll
    for (int j = 0; j < DPL; ++j)
      if (has_obst[j]) {
        s_eprev[lane + j * LPE] = ego_obst(my[j], x0, y0, c0, s0);
        if (cfg.moving) move_obstacle(cfg, my[j]);
      }
    t = t + 1;
    // ---- velocity (train.py:182-188): per-step displacement ----
    const double ddx = x1 - x0, ddy = y1 - y0;
    vlin = sqrt(ddx * ddx + ddy * ddy);
    vang = pi_to_pi(yaw1 - yaw0);
    t_obs = (float)cfg.dt;
  }
  FFMP_ENV_STAMP(1);

#pragma unroll
  for (int j = 0; j < DPL; ++j)
    if (has_obst[j]) lidar_disc(x1, y1, my[j].x, my[j].y, my[j].r, s_ox, s_oy, s_orr, s_or, lane + j * LPE);
  double c1 = cos(yaw1), s1 = sin(yaw1);
  float4 ecur1[DPL];
#pragma unroll
  for (int j = 0; j < DPL; ++j) {
    ecur1[j] = has_obst[j] ? ego_obst(my[j], x1, y1, c1, s1) : make_float4(0.f, 0.f, 0.f, 0.f);
    if (has_obst[j]) s_ecur[lane + j * LPE] = ecur1[j];
  }
  wave_sync();

  FFMP_ENV_STAMP(2);
  FrameHdr hcur = make_hdr(x1, y1, c1, s1);
  FrameHdr hprev = (MODE == kEnvMode_Step) ? make_hdr(x0, y0, c0, s0) : hcur;

  // ---- the env's outputs from its post-step state: field gradient at the robot cell (central
  // differences), raster record, state write-back, small obs.  Round 4: a stepped env runs this
  // BEFORE its lidar and collision tests — nothing here depends on them — and an env that then
  // resets runs it again for its new episode (first = 1) over what it wrote: the lidar's float64
  // chains no longer keep the whole post-step state live (fewer registers), and the bytes
  // written are the same. ----
  auto finish = [&](bool first) {
    const float2 ge = to_ego(gx, gy, x1, y1, c1, s1);
    float U = 0.0f;
    if (lane < 4) {
      const int di = (lane == 0) ? 1 : (lane == 1) ? -1 : 0;
      const int dj = (lane == 2) ? 1 : (lane == 3) ? -1 : 0;
      U = potential_cell(cfg, s_ecur, K, ge.x, ge.y, ic + di, ic + dj);
    }
    const float Uxp = __shfl(U, 0, LPE), Uxm = __shfl(U, 1, LPE), Uyp = __shfl(U, 2, LPE),
                Uym = __shfl(U, 3, LPE);
    if (lane == 0) {
      ob.grad[e * 2 + 0] = (Uxp - Uxm) * cfg.inv_2res_f;
      ob.grad[e * 2 + 1] = (Uyp - Uym) * cfg.inv_2res_f;
    }
    float* rec = st.record + e * rec_stride(K);
    // the terminal state (keep_terminal): the post-step record of a stepped env — also when it
    // resets below, which rewrites only st.record
    float* term = (MODE == kEnvMode_Step && !first && st.term_record) ? st.term_record + e * rec_stride(K) : nullptr;
    write_record_hdr(rec, lane, hcur, hprev, ge, first ? 1.0f : 0.0f);
    if (term) write_record_hdr(term, lane, hcur, hprev, ge, 0.0f);
#pragma unroll
    for (int j = 0; j < DPL; ++j) {
      if (!has_obst[j]) continue;
      const int k = lane + j * LPE;
      const float4 ecur = s_ecur[k], eprev = s_eprev[k];
      const float4 vel = ego_vel(my[j], c1, s1);
      write_record_obst(rec, k, K, ecur, eprev, vel);
      if (term) write_record_obst(term, k, K, ecur, eprev, vel);
      if (s_rvel) s_rvel[k] = make_float2(vel.x, vel.y);
      double* p = st.obst + (e * K + k) * 4;
      p[0] = my[j].x; p[1] = my[j].y; p[2] = my[j].vx; p[3] = my[j].vy;
      st.obst_r[e * K + k] = my[j].r;
    }
    if (s_rhdr) {  // the one-launch step: the record's header for the block's raster, in LDS
      if (lane < FFMP_REC_HDR) {
        const float hv[FFMP_REC_HDR] = {hcur.px, hcur.py, hcur.c, hcur.s, hprev.px, hprev.py, hprev.c, hprev.s,
                                        ge.x,    ge.y,    first ? 1.0f : 0.0f, 0.0f, 0.0f, 0.0f, 0.0f, 0.0f};
        s_rhdr[lane] = hv[lane];
      }
    }
    if (lane == 0) {
      st.pose[e * 3 + 0] = x1; st.pose[e * 3 + 1] = y1; st.pose[e * 3 + 2] = yaw1;
      st.goal[e * 2 + 0] = gx; st.goal[e * 2 + 1] = gy;
      st.d0[e] = d0;
      st.t[e] = t;
      st.episode[e] = episode;
      ob.state_v[e * 2 + 0] = (float)vlin;
      ob.state_v[e * 2 + 1] = (float)vang;
      ob.state_t[e] = t_obs;
    }
  };

  if (MODE == kEnvMode_Step) {
    // ---- relative goal (train.py:174-180) ----
    const double dx = gx - x1, dy = gy - y1;
    const double dist = sqrt(dx * dx + dy * dy);
    if (lane == 0) {
      // small obs of the post-step state (a reset below overwrites state_g)
      const float g0 = (float)dist, g1 = (float)pi_to_pi(atan2(dy, dx) - yaw1);
      ob.state_g[e * 2 + 0] = g0;
      ob.state_g[e * 2 + 1] = g1;
      if (st.term_obs) {
        float* to = st.term_obs + e * 5;
        to[0] = g0; to[1] = g1; to[2] = (float)vlin; to[3] = (float)vang; to[4] = t_obs;
      }
    }
    finish(false);
    FFMP_ENV_STAMP(3);
    // ---- collision: footprint on the current occupancy (ffmp.py:85-105) ----
    // (cells in a wave-uniform loop over the offsets staged in LDS by stage_footprint, discs
    // lane-parallel: lane k tests its disc k, lane 0 the walls; the ballot below ORs them:
    // occupied_cell's value for every cell)
    // (round 4) Most waves skip the loop: with the cells' extent fb = {max |ex|, max |ey|}, a disc
    // whose centre is farther than r (+ 0.01 % + 1 um) beyond it along x or y contains no cell
    // (|ex - ox| > r, so (ex - ox)^2 > r^2 after rounding), and a robot farther than the cells' reach
    // (+ margins) from every wall has no cell outside the world (|c ex - s ey| <= |ex| + |ey|): the
    // loop would return false.  Collisions are rare, so the test runs only where one is possible.
    bool c_foot = false;
    if (cfg.collide_mode & FFMP_COLLIDE_FOOTPRINT) {
      const float2 fb = s_foot[FFMP_MAX_FOOT];
      const float Wf = cfg.world_half_f * 0.9999f, reach = (fb.x + fb.y) * 1.0001f + 1e-6f;
      const bool wall = !(fabsf(hcur.px) + reach < Wf && fabsf(hcur.py) + reach < Wf);
      bool disc[DPL], anyd = false;
#pragma unroll
      for (int j = 0; j < DPL; ++j) {
        const float rr = ecur1[j].w * 1.0001f + 1e-6f;
        disc[j] = has_obst[j] && !(fabsf(ecur1[j].x) - fb.x > rr || fabsf(ecur1[j].y) - fb.y > rr);
        anyd = anyd || disc[j];
      }
      if (__ballot(anyd || (wall && lane == 0)) != 0) {
        for (int f = 0; f < cfg.n_foot; ++f) {
          const float2 fc = s_foot[f];
          const float ex = fc.x, ey = fc.y;
          bool hit = wall && lane == 0 && outside_world(cfg, hcur, ex, ey);
#pragma unroll
          for (int j = 0; j < DPL; ++j) hit = hit || (disc[j] && in_disc(ex, ey, ecur1[j]));
          c_foot |= hit;
        }
      }
    }
    FFMP_ENV_STAMP(7);
    // ---- lidar + is_collision2 (ffmp.py:108-117) ----
    bool c_lidar = false;
    const LidarScene sc = lidar_scene<DPL>(cfg, x1, y1, my, lane, K, LPE);
    if constexpr (DL) {
      trace_discs<DPL>(cfg, sc, lane, LPE, x1, y1, c1, s1, s_ox, s_oy, s_orr, s_or, s_key, s_pref, s_lo, [&](int l, double r) {
        const float rf = (float)r;
        ob.lidar[e * L + l] = rf;
        c_lidar |= beam_collides(rf, cfg.robot_r);
      });
    } else if constexpr (BCH > 1) {
      trace_beams<BCH>(cfg, sc, lane, LPE, x1, y1, c1, s1, s_ox, s_oy, s_orr, s_or, [&](int l, double r) {
        const float rf = (float)r;
        ob.lidar[e * L + l] = rf;
        c_lidar |= beam_collides(rf, cfg.robot_r);
      });
    } else {
      for_beams(cfg, lane, LPE, beam0, [&](int l, double2 b) {
        const float rf = (float)lidar_beam(cfg, sc, x1, y1, c1, s1, b.x, b.y, s_ox, s_oy, s_orr, s_or);
        ob.lidar[e * L + l] = rf;
        c_lidar |= beam_collides(rf, cfg.robot_r);
      });
    }
    FFMP_ENV_STAMP(8);
    c_foot = group_ballot(c_foot, LPE) != 0;
    c_lidar = (group_ballot(c_lidar, LPE) != 0) && (cfg.collide_mode & FFMP_COLLIDE_LIDAR);
    // ---- is_goal / reward / is_done (ffmp.py:120-164), truncation (train.py:607) ----
    const bool col = c_foot || c_lidar;
    const bool goal = dist < cfg.goal_thr;
    const double reward = reward_calc(dist, d0, col, goal);
    const bool trunc = (cfg.max_steps > 0) && (t >= cfg.max_steps);
    const bool done = col || goal || trunc;
    reset_now = done && cfg.autoreset;
    if (lane == 0) {
      out.reward[e] = (float)reward;
      out.done[e] = done;
      out.is_goal[e] = goal;
      out.collide[e] = col;
      out.truncated[e] = trunc;
    }
    FFMP_ENV_STAMP(9);
  }

  FFMP_ENV_STAMP(4);
  if (reset_now) {
    // ---- episode reset (the external /episode_manager; train.py:559-566) ----
    episode = (MODE == kEnvMode_Reset && initial) ? 0 : episode + 1;
    const Episode ep = sample_episode(cfg, genv, episode);
    x1 = ep.x; y1 = ep.y; yaw1 = ep.yaw; gx = ep.gx; gy = ep.gy;
    wave_sync();  // all lanes done reading the terminal-state LDS arrays
#pragma unroll
    for (int j = 0; j < DPL; ++j)
      if (has_obst[j]) my[j] = sample_obstacle(cfg, genv, episode, lane + j * LPE, ep);
    c1 = cos(yaw1); s1 = sin(yaw1);
#pragma unroll
    for (int j = 0; j < DPL; ++j)
      if (has_obst[j]) {
        const int k = lane + j * LPE;
        lidar_disc(x1, y1, my[j].x, my[j].y, my[j].r, s_ox, s_oy, s_orr, s_or, k);
        const float4 eo = ego_obst(my[j], x1, y1, c1, s1);
        s_ecur[k] = eo;
        s_eprev[k] = eo;  // temporal stack duplicated on the first step (train.py:475-478)
      }
    wave_sync();
    hcur = make_hdr(x1, y1, c1, s1);
    hprev = hcur;
    t = 0;
    vlin = 0.0; vang = 0.0;  // robot_velocity_calculator with is_first (train.py:183-184)
    t_obs = 0.0f;            // odom dt on the first step (train.py:532-533,540)
    const double dx = gx - x1, dy = gy - y1;
    const double dist = sqrt(dx * dx + dy * dy);
    d0 = dist;  // pre_relative_goal_dist on is_first (ffmp.py:139-141)
    if (lane == 0) {
      ob.state_g[e * 2 + 0] = (float)dist;
      ob.state_g[e * 2 + 1] = (float)pi_to_pi(atan2(dy, dx) - yaw1);
    }
    const LidarScene sc = lidar_scene<DPL>(cfg, x1, y1, my, lane, K, LPE);
    if constexpr (DL) {
      trace_discs<DPL>(cfg, sc, lane, LPE, x1, y1, c1, s1, s_ox, s_oy, s_orr, s_or, s_key, s_pref, s_lo,
                  [&](int l, double r) { ob.lidar[e * L + l] = (float)r; });
    } else if constexpr (BCH > 1) {
      trace_beams<BCH>(cfg, sc, lane, LPE, x1, y1, c1, s1, s_ox, s_oy, s_orr, s_or,
                                   [&](int l, double r) { ob.lidar[e * L + l] = (float)r; });
    } else {
      for_beams(cfg, lane, LPE, beam0, [&](int l, double2 b) {
        ob.lidar[e * L + l] = (float)lidar_beam(cfg, sc, x1, y1, c1, s1, b.x, b.y, s_ox, s_oy, s_orr, s_or);
      });
    }
    finish(true);
  }
  FFMP_ENV_STAMP(6);
}

// FFMP_ENV_WPE: a probe knob (tools/ builds) — ask the compiler for at least this many waves per SIMD
#ifdef FFMP_ENV_WPE
#define FFMP_ENV_OCC __attribute__((amdgpu_waves_per_eu(FFMP_ENV_WPE)))
#else
#define FFMP_ENV_OCC
#endif
template <int MODE, int kEnvWaves, int LPE, int DPL>
__global__ __launch_bounds__(64 * kEnvWaves) FFMP_ENV_OCC void env_kernel(ffmp_cfg_t cfg, int64_t n, int64_t env_offset,
                                                 const int64_t* __restrict__ action,
                                                 const uint8_t* __restrict__ mask, int32_t initial,
                                                 ffmp_state_t st, ffmp_obs_t ob, ffmp_out_t out) {
  constexpr int EPW = 64 / LPE;  // envs per wave
  constexpr int DS = 64 * DPL;    // disc slots per wave: EPW envs x LPE lanes x DPL discs
  __shared__ double s_oxa[kEnvWaves][DS], s_oya[kEnvWaves][DS], s_ora[kEnvWaves][DS], s_orra[kEnvWaves][DS];
  __shared__ float4 s_ecura[kEnvWaves][DS], s_epreva[kEnvWaves][DS];
  __shared__ float2 s_foota[kEnvWaves][FFMP_MAX_FOOT + 1];  // + the cells' extent
  // the disc-major lidar's per-env beam minima ([wave][env][L] uint32, dynamic: L * 4 bytes per env)
  // and per-disc pair counts / first beams
  extern __shared__ uint32_t s_keys[];
  __shared__ int s_prefa[kEnvWaves][DS], s_loa[kEnvWaves][DS];

  const int wv = threadIdx.x >> 6;
  const int grp = (threadIdx.x & 63) / LPE;
  const int64_t e = ((int64_t)blockIdx.x * kEnvWaves + wv) * EPW + grp;
  const int lane = threadIdx.x & (LPE - 1);  // lane within the env's group
  if (MODE == kEnvMode_Step) stage_footprint(cfg, s_foota[wv]);
  if (e >= n) return;
  if (MODE == kEnvMode_Reset && mask && !mask[e]) return;
  const int g0 = grp * LPE * DPL;  // the env's disc slots
  env_group<MODE, LPE, FFMP_BEAM_CHUNK, true, DPL>(cfg, env_offset, action, initial, st, ob, out, e, lane,
                       s_oxa[wv] + g0, s_oya[wv] + g0, s_ora[wv] + g0, s_orra[wv] + g0,
                       s_ecura[wv] + g0, s_epreva[wv] + g0, s_foota[wv], nullptr, nullptr,
                       s_keys + ((size_t)wv * EPW + grp) * cfg.n_beams, s_prefa[wv] + g0, s_loa[wv] + g0);
}

// ============================================================================
// raster_kernel: the HBM-bound hot path.
//   block = 256 threads (4 waves); a pass covers 1024 consecutive cells of one
//   env plane (each wave a contiguous 256-cell chunk, each lane 4 cells = one
//   16-B store per plane).  Obstacles of both frames sit in LDS and lane k keeps
//   obstacle k in registers; per chunk the cull is lane-parallel (lane k tests
//   obstacle k against the chunk's ego bounding box, one __ballot builds the
//   wave-uniform mask), and lanes 0..7 test the chunk corners against the world
//   walls the same way, so the per-cell wall test runs only near a wall.
// ============================================================================
namespace {

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <bool NT>
FFMP_DEV void store4(float* p, float a, float b, float c, float d) {
  f32x4 v = {a, b, c, d};
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(p));
  else *reinterpret_cast<f32x4*>(p) = v;
}

// Compact observation format (FFMP_OBS_U8F16): a lane's 4 occupancy cells as 4 bytes (0 / 255)
// in one dword store, its 4 potential cells as binary16 (round to nearest even, as numpy's
// float32 -> float16 cast) in one dwordx2 store.
FFMP_DEV uint32_t pack4_u8(const float occ[4]);

template <bool NT>
FFMP_DEV void store4_u8(uint8_t* p, const float occ[4]) {
  const uint32_t v = pack4_u8(occ);
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<uint32_t*>(p));
  else *reinterpret_cast<uint32_t*>(p) = v;
}

typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

FFMP_DEV uint32_t pack4_u8(const float occ[4]) {
  return (occ[0] != 0.0f ? 0xFFu : 0u) | (occ[1] != 0.0f ? 0xFF00u : 0u) | (occ[2] != 0.0f ? 0xFF0000u : 0u) |
         (occ[3] != 0.0f ? 0xFF000000u : 0u);
}

// 16 cells of a lane as one 16-B store (the frame) and two 16-B stores (the potential): whole
// 16-B lane segments, as the float32 layout's, so nontemporal stores stay full-width
template <bool NT>
FFMP_DEV void store16_u8(uint8_t* p, const float occ[16]) {
  u32x4 v = {pack4_u8(occ), pack4_u8(occ + 4), pack4_u8(occ + 8), pack4_u8(occ + 12)};
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = v;
}

// 8 cells of a lane as one 8-B frame store
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <bool NT>
FFMP_DEV void store8_u8(uint8_t* p, const float occ[8]) {
  u32x2 v = {pack4_u8(occ), pack4_u8(occ + 4)};
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x2*>(p));
  else *reinterpret_cast<u32x2*>(p) = v;
}

template <bool NT>
FFMP_DEV void store8_h(_Float16* p, const float* U) {
  f16x8 v = {(_Float16)U[0], (_Float16)U[1], (_Float16)U[2], (_Float16)U[3],
             (_Float16)U[4], (_Float16)U[5], (_Float16)U[6], (_Float16)U[7]};
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<f16x8*>(p));
  else *reinterpret_cast<f16x8*>(p) = v;
}

// 16 occupancy bytes already packed as 4 words (0x00 / 0xFF per byte) as one 16-B store
template <bool NT>
FFMP_DEV void store16_w(uint8_t* p, const uint32_t w[4]) {
  u32x4 v = {w[0], w[1], w[2], w[3]};
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(p));
  else *reinterpret_cast<u32x4*>(p) = v;
}

template <bool NT>
FFMP_DEV void store4_h(_Float16* p, float a, float b, float c, float d) {
  f16x4 v = {(_Float16)a, (_Float16)b, (_Float16)c, (_Float16)d};
  if (NT) __builtin_nontemporal_store(v, reinterpret_cast<f16x4*>(p));
  else *reinterpret_cast<f16x4*>(p) = v;
}

// A wave-uniform float moved to a scalar register.
FFMP_DEV float uni(float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); }

FFMP_DEV float box_dist2(float px, float py, float x0, float x1, float y0, float y1) {
  const float dx = fmaxf(fmaxf(x0 - px, px - x1), 0.0f);
  const float dy = fmaxf(fmaxf(y0 - py, py - y1), 0.0f);
  return dx * dx + dy * dy;
}

FFMP_DEV bool corner_inside(const ffmp_cfg_t& cfg, const FrameHdr& h, float ex, float ey) {
  const float wx = h.px + (h.c * ex - h.s * ey);
  const float wy = h.py + (h.s * ex + h.c * ey);
  const float W = cfg.world_half_f - cfg.cull_margin_f;
  return (fabsf(wx) <= W) && (fabsf(wy) <= W);
}

// r / G for 0 <= r < 1024 + G (8 <= G <= 4096): (r + 0.5) / G is >= 0.5/G away
// from an integer, far more than the float32 error of the product.
FFMP_DEV int small_div(int r, float invG) { return (int)(((float)r + 0.5f) * invG); }

}  // namespace

// XCD-aware remap: blocks are dealt round-robin over the 8 XCDs (b and b+8 share one), so
// logical block (b % 8) * per + b / 8 gives every XCD a contiguous range of (env, tile) work:
// 8x less concurrently written footprint per XCD.  A placement-only change.
template <bool XCD>
FFMP_DEV int64_t logical_block() {
  int64_t lb = blockIdx.x;
  if (XCD) {
    const int64_t per = (int64_t)gridDim.x / 8;
    if (lb < per * 8) lb = (lb % 8) * per + lb / 8;
  }
  return lb;
}


// Observation format of a raster instantiation: FMT_F32 (reference layout), FMT_CT4 (compact
// FFMP_OBS_U8F16, 4 cells per lane) or FMT_CT16 (compact, 16 cells per lane: a wave task is
// 1024 cells, so the per-task cull / wall / index work is spread over 4x the cells — the compact
// raster writes 3 bytes per cell and is bound by that per-task work, not by HBM; needs G % 16 == 0).
// FMT_CT8 (FFMP_RASTER_MID8, G % 8 == 0): 8 cells per lane, an 8-B frame store and a 16-B potential
// store per lane (512-cell wave tasks).
constexpr int FMT_F32 = 0, FMT_CT4 = 1, FMT_CT16 = 2, FMT_CT8 = 3;
// The CT8 raster is held to 6 waves per SIMD (84 VGPRs instead of the compiler's 112 at 4): C3
// newest-only raster 0.985-1.025 -> 0.954-0.956 ms (profiles/r03b_ct8_shapes.txt).
#ifndef FFMP_CT8_MIN_WAVES
#define FFMP_CT8_MIN_WAVES 6
#endif

// The raster of cells [tile * cells_per_block, ...) of env e by the whole 256-thread block
// (block-uniform arguments; contains a block barrier).  Compact formats: state_m holds uint8
// frames and pot binary16 planes (the pointers are reinterpreted; strides in elements).
// PRELOADED: the record is already in the block's LDS (s_hdr, s_cur, s_prev, s_vel; written by the
// one-launch step's env_group before a block barrier), so the raster does not read it back from HBM.
template <bool NT, bool FLOW, int FMT, bool PRELOADED = false>
FFMP_DEV __attribute__((always_inline)) void raster_env(const ffmp_cfg_t& cfg, int64_t e, int tile, int32_t cells_per_block,
                                                        const float* __restrict__ record,
                                                        float* __restrict__ state_m, int64_t sm_stride,
                                                        int64_t sm_frame, int32_t newest_only,
                                                        float* __restrict__ pot, float* __restrict__ flow,
                                                        int32_t tile_log2r, float4* s_cur, float4* s_prev,
                                                        float2* s_vel, float* s_hdr) {
  constexpr bool CT = FMT != FMT_F32;
  constexpr int CPL = FMT == FMT_CT16 ? 16 : FMT == FMT_CT8 ? 8 : 4;  // cells per lane in a wave task
  constexpr int WC = 64 * CPL;                   // cells per wave task
  const int K = cfg.n_obst;
  const int G = cfg.grid;
  const int G2 = G * G;
  const int tid = threadIdx.x;
  if (!PRELOADED) FFMP_RAS_STAMP(0);
  const float* rec = record + e * rec_stride(K);
  if (!PRELOADED) {
    if (tid < FFMP_REC_HDR) s_hdr[tid] = rec[tid];
    if (tid < K) {
      const float* ro = rec + FFMP_REC_HDR;  // 4-B words: the ABI asks no more alignment of the record
      const float* c = ro + 4 * tid;
      const float* q = ro + 4 * (K + tid);
      s_cur[tid] = make_float4(c[0], c[1], c[2], c[3]);
      s_prev[tid] = make_float4(q[0], q[1], q[2], q[3]);
      if (FLOW) s_vel[tid] = make_float2(ro[4 * (2 * K + tid)], ro[4 * (2 * K + tid) + 1]);
    }
    __syncthreads();
  }
  if (!PRELOADED) FFMP_RAS_STAMP(1);

  // The header is block-uniform.  FMT_CT4: keep it in scalar registers (readfirstlane) instead of
  // 11 VGPRs — 108 -> 72 VGPRs, 4 -> 7 waves per SIMD, compact C3 raster 1.15-1.29 -> 1.00-1.13 ms
  // (profiles/r02_occupancy.txt).  Not for the float32 layout (store-bound: 7 waves per SIMD ran
  // its steps ~2 % slower than 4) nor for FMT_CT16 (the scheduler then took 188 VGPRs, not 167).
  auto hv = [&](int i) { return (FMT == FMT_CT4 || FMT == FMT_CT8) ? uni(s_hdr[i]) : s_hdr[i]; };
  const FrameHdr hc{hv(0), hv(1), hv(2), hv(3)};
  const FrameHdr hp{hv(4), hv(5), hv(6), hv(7)};
  const float gx = hv(8), gy = hv(9);
  // temporal stack in place: the older frame already holds the previous newest one unless this
  // env was reset (block-uniform)
  const bool write_old = !newest_only || hv(10) != 0.0f;
  const float res = cfg.res_f, half = cfg.half_f;
  const float invG = 1.0f / (float)G;

  const int wave = tid >> 6, lane = tid & 63;
  // lane k's obstacle (cull operand) and its squared reach
  const bool has = lane < K;
  const float4 oc = has ? s_cur[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  const float4 op = has ? s_prev[lane] : make_float4(0.f, 0.f, 0.f, 0.f);
  const bool with_pot = pot != nullptr;  // uniform: skip the potential entirely without a plane
  // potential reach (covers occupancy), or the occupancy reach alone without a potential plane
  const float rc = oc.w + (with_pot ? cfg.rho0_f : 0.0f) + cfg.cull_margin_f;
  const float rp = op.w + cfg.cull_margin_f;               // occupancy reach
  const float rc2 = rc * rc, rp2 = rp * rp;
  // lanes 0..3: corners of the current frame, 4..7: previous frame
  const FrameHdr hq = (lane < 4) ? hc : hp;

  float* m0 = state_m + e * sm_stride;
  float* m1 = m0 + sm_frame;
  float* pp = pot ? pot + (int64_t)e * G2 : nullptr;
  uint8_t* b0 = CT ? reinterpret_cast<uint8_t*>(state_m) + e * sm_stride : nullptr;
  uint8_t* b1 = CT ? b0 + sm_frame : nullptr;
  _Float16* hp16 = (CT && pot) ? reinterpret_cast<_Float16*>(pot) + (int64_t)e * G2 : nullptr;
  float* f0 = (FLOW && !CT) ? flow + (int64_t)e * 2 * G2 : nullptr;
  _Float16* h0 = (FLOW && CT) ? reinterpret_cast<_Float16*>(flow) + (int64_t)e * 2 * G2 : nullptr;  // binary16 flow

  const int qbeg = tile * cells_per_block;
  const int qend = min(qbeg + cells_per_block, G2);

  // One wave task: the cells of ego rows [i0, i1] x columns [j0, j1] (the cull box), this
  // lane's CPL cells (i, j..j+CPL-1) at plane offset q, `valid` = the lane has cells.
  auto task = [&](int i0, int i1, int j0, int j1, int i, int j, int q, bool valid) {
    const float bx0 = (float)i0 * res - half, bx1 = (float)i1 * res - half;
    const float by0 = (float)j0 * res - half, by1 = (float)j1 * res - half;

    // ---- lane-parallel cull ----
    const uint64_t mc = __ballot(has && box_dist2(oc.x, oc.y, bx0, bx1, by0, by1) <= rc2);
    const uint64_t mp = write_old ? __ballot(has && box_dist2(op.x, op.y, bx0, bx1, by0, by1) <= rp2) : 0ull;
    const uint64_t wb = __ballot(lane >= 8 || corner_inside(cfg, hq, (lane & 1) ? bx1 : bx0,
                                                             (lane & 2) ? by1 : by0));
    const bool walls_c = (wb & 0xFull) != 0xFull;
    const bool walls_p = write_old && (wb & 0xF0ull) != 0xF0ull;
    if (!valid) return;

    // ---- this lane's CPL cells ----
    const float ex = (float)i * res - half;
    float ey[CPL];
#pragma unroll
    for (int u = 0; u < CPL; ++u) ey[u] = (float)(j + u) * res - half;

    float occp[CPL], occc[CPL], U[CPL];
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
      occp[u] = (walls_p && outside_world(cfg, hp, ex, ey[u])) ? 1.0f : 0.0f;
      occc[u] = (walls_c && outside_world(cfg, hc, ex, ey[u])) ? 1.0f : 0.0f;
      U[u] = with_pot ? attractive(cfg, ex, ey[u], gx, gy) : 0.0f;
    }
    for (uint64_t m = mp; m; m &= m - 1) {
      const float4 o = s_prev[__builtin_ctzll(m)];
#pragma unroll
      for (int u = 0; u < CPL; ++u) if (in_disc(ex, ey[u], o)) occp[u] = 1.0f;
    }
    float fx[CPL], fy[CPL];
    bool fset[CPL];
#pragma unroll
    for (int u = 0; u < CPL; ++u) {
      fx[u] = fy[u] = 0.0f;
      fset[u] = false;
    }
    for (uint64_t m = mc; m; m &= m - 1) {
      const int k = __builtin_ctzll(m);
      const float4 o = s_cur[k];
      const float reach2 = rep_reach2(cfg, o.w);
      const float dx = ex - o.x;
#pragma unroll
      for (int u = 0; u < CPL; ++u) {
        const float dy = ey[u] - o.y;
        const float d2 = dx * dx + dy * dy;  // in_disc's and add_repulsive's operand
        const bool d = d2 <= o.z;
        if (d) occc[u] = 1.0f;
        if (FLOW && d && !fset[u]) {  // lowest disc index covering the cell
          fx[u] = s_vel[k].x;
          fy[u] = s_vel[k].y;
          fset[u] = true;
        }
        if (with_pot) U[u] = add_repulsive_s(cfg, U[u], d2, o.w, reach2);
      }
    }
    if (CT && CPL == 16) {
      if (write_old) store16_u8<NT>(b0 + q, occp);
      store16_u8<NT>(b1 + q, occc);
      if (hp16) {
        store8_h<NT>(hp16 + q, U);
        store8_h<NT>(hp16 + q + 8, U + 8);
      }
      if (FLOW) {
        store8_h<NT>(h0 + q, fx);
        store8_h<NT>(h0 + q + 8, fx + 8 % CPL);
        store8_h<NT>(h0 + G2 + q, fy);
        store8_h<NT>(h0 + G2 + q + 8, fy + 8 % CPL);
      }
      return;
    }
    if constexpr (CT && CPL == 8) {
      if (write_old) store8_u8<NT>(b0 + q, occp);
      store8_u8<NT>(b1 + q, occc);
      if (hp16) store8_h<NT>(hp16 + q, U);
      if (FLOW) {
        store8_h<NT>(h0 + q, fx);
        store8_h<NT>(h0 + G2 + q, fy);
      }
      return;
    }
    if (CT) {
      if (write_old) store4_u8<NT>(b0 + q, occp);
      store4_u8<NT>(b1 + q, occc);
      if (hp16) store4_h<NT>(hp16 + q, U[0], U[1], U[2], U[3]);
      if (FLOW) {
        store4_h<NT>(h0 + q, fx[0], fx[1], fx[2], fx[3]);
        store4_h<NT>(h0 + G2 + q, fy[0], fy[1], fy[2], fy[3]);
      }
      return;
    }
    if (write_old) store4<NT>(m0 + q, occp[0] * 255.0f, occp[1] * 255.0f, occp[2] * 255.0f, occp[3] * 255.0f);
    store4<NT>(m1 + q, occc[0] * 255.0f, occc[1] * 255.0f, occc[2] * 255.0f, occc[3] * 255.0f);
    if (pp) store4<NT>(pp + q, U[0], U[1], U[2], U[3]);
    if (FLOW) {
      store4<NT>(f0 + q, fx[0], fx[1], fx[2], fx[3]);
      store4<NT>(f0 + G2 + q, fy[0], fy[1], fy[2], fy[3]);
    }
  };

  if (tile_log2r > 0) {
    // 2-D wave tiles of R rows x C = WC/R columns (the host checked G % C == 0 and that the
    // block holds whole bands of R rows): a compact cull box (C3, R = 4: 0.2 m x 3.2 m instead
    // of one 12.8 m row), so far fewer discs survive the cull; every row segment is C cells
    // of contiguous, 4*CPL-byte-per-lane (float32) stores.  Tiles are dealt band-major to the 4
    // waves, so the waves of a block write neighbouring columns of the same rows at once.
    const int R = 1 << tile_log2r, C = WC >> tile_log2r;
    const int lanes_per_row = 64 >> tile_log2r;
    const int ncb = G / C;
    const int row0 = qbeg / G;
    const int ntiles = ((qend - qbeg) / G / R) * ncb;
    const int r = lane / lanes_per_row;
    const int cl = (lane - r * lanes_per_row) * CPL;
    if ((4 % ncb) == 0 || (ncb % 4) == 0) {
      // Column-band-major tiles: wave w takes column bands w, w + 4, ... (ncb >= 4) or the
      // bands b = w / ncb, + 4 / ncb, ... of column band w % ncb (ncb | 4), so per column band
      // this lane's CPL columns, their ego y and (y - goal y)^2 are computed once instead of per
      // tile (the 4 waves still write neighbouring columns of the same rows at once), the attractive
      // term is then one add + one multiply per cell (packed pairs), and the occupancy is kept as
      // the stored bytes (0x00 / 0xFF; float32: v_cvt_f32_ubyte gives 0 / 255) instead of floats.
      // The same float32 operations in the same order as `task`: bit-identical planes.  (Round 2:
      // the compact raster's VALU instructions per launch 1.02e9 -> 0.42e9, profiles/r02_compact.txt.)
      typedef float f2 __attribute__((ext_vector_type(2)));
      constexpr int NP = CPL / 2, NW = CPL / 4;
      const int nbands = ntiles / ncb;
      const int wpc = ncb < 4 ? 4 / ncb : 1;  // waves per column band
      const f2 hka = {cfg.half_ka_f, cfg.half_ka_f};
      for (int cb = wave % ncb; cb < ncb; cb += 4) {
        const int jb = cb * C, j = jb + cl;
        const float by0 = (float)jb * res - half, by1 = (float)(jb + C - 1) * res - half;
        // the cull's column-band part per lane (disc): what is left of the reach^2 for the row
        // distance, so a band's test is dx^2 <= tc — the same box test as box_dist2 <= rc2 up to
        // float rounding (~1e-7 of rc^2), which the cull margin (0.1 m, i.e. ~0.1 of rc^2) covers
        // many times over: culling stays conservative.  One VGPR per frame instead of the reach^2
        // and the column term (the loop had spilled those and, reloading them, waited for every
        // store of the previous band: vmcnt(0))
        const float dyc = fmaxf(fmaxf(by0 - oc.y, oc.y - by1), 0.0f);
        const float dyp = fmaxf(fmaxf(by0 - op.y, op.y - by1), 0.0f);
        const float tc = rc2 - dyc * dyc, tp = rp2 - dyp * dyp;
        f2 ey2[NP], dyy2[NP];
#pragma unroll
        for (int p2 = 0; p2 < NP; ++p2) {
          ey2[p2] = f2{(float)(j + 2 * p2) * res - half, (float)(j + 2 * p2 + 1) * res - half};
          const f2 dy = ey2[p2] - gy;
          dyy2[p2] = dy * dy;
        }
        for (int band = wave / ncb; band < nbands; band += wpc) {
          const int i0 = row0 + band * R;
          const int i = i0 + r;
          const int q = i * G + j;
          const float bx0 = (float)i0 * res - half, bx1 = (float)(i0 + R - 1) * res - half;
          const float dxc = fmaxf(fmaxf(bx0 - oc.x, oc.x - bx1), 0.0f);
          const uint64_t mc = __ballot(has && dxc * dxc <= tc);
          uint64_t mp = 0ull;
          if (write_old) {
            const float dxp = fmaxf(fmaxf(bx0 - op.x, op.x - bx1), 0.0f);
            mp = __ballot(has && dxp * dxp <= tp);
          }
          const uint64_t wb = __ballot(lane >= 8 || corner_inside(cfg, hq, (lane & 1) ? bx1 : bx0,
                                                                   (lane & 2) ? by1 : by0));
          const bool walls_c = (wb & 0xFull) != 0xFull;
          const bool walls_p = write_old && (wb & 0xF0ull) != 0xF0ull;
          const float ex = (float)i * res - half;
          uint32_t wc[NW], wp[NW];
#pragma unroll
          for (int w = 0; w < NW; ++w) wc[w] = wp[w] = 0u;
          f2 U2[NP];
          if (with_pot) {
            const float dx = ex - gx;
            const f2 dxx = {dx * dx, dx * dx};
#pragma unroll
            for (int p2 = 0; p2 < NP; ++p2) U2[p2] = hka * (dxx + dyy2[p2]);
          }
          if (walls_c) {
#pragma unroll
            for (int u = 0; u < CPL; ++u)
              if (outside_world(cfg, hc, ex, ey2[u >> 1][u & 1])) wc[u >> 2] |= 0xFFu << (8 * (u & 3));
          }
          if (walls_p) {
#pragma unroll
            for (int u = 0; u < CPL; ++u)
              if (outside_world(cfg, hp, ex, ey2[u >> 1][u & 1])) wp[u >> 2] |= 0xFFu << (8 * (u & 3));
          }
          for (uint64_t m = mp; m; m &= m - 1) {
            const float4 o = s_prev[__builtin_ctzll(m)];
#pragma unroll
            for (int u = 0; u < CPL; ++u)
              if (in_disc(ex, ey2[u >> 1][u & 1], o)) wp[u >> 2] |= 0xFFu << (8 * (u & 3));
          }
          float fx[FLOW ? CPL : 1], fy[FLOW ? CPL : 1];
          uint32_t fset = 0u;  // FLOW: cells already covered by a lower-index disc
          if (FLOW) {
#pragma unroll
            for (int u = 0; u < CPL; ++u) fx[u] = fy[u] = 0.0f;
          }
          for (uint64_t m = mc; m; m &= m - 1) {
            const int k = __builtin_ctzll(m);
            const float4 o = s_cur[k];
            const float reach2 = rep_reach2(cfg, o.w);
            const float dx = ex - o.x;
            const f2 dxx = {dx * dx, dx * dx};
#pragma unroll
            for (int p2 = 0; p2 < NP; ++p2) {
              const f2 dy = ey2[p2] - o.y;
              const f2 d2 = dxx + dy * dy;  // in_disc's and add_repulsive's operand
#pragma unroll
              for (int c = 0; c < 2; ++c) {
                const int u = 2 * p2 + c;
                const bool d = d2[c] <= o.z;
                if (d) wc[u >> 2] |= 0xFFu << (8 * (u & 3));
                if (FLOW && d && !((fset >> u) & 1u)) {
                  fx[u] = s_vel[k].x;
                  fy[u] = s_vel[k].y;
                  fset |= 1u << u;
                }
                if (with_pot) U2[p2][c] = add_repulsive_s(cfg, U2[p2][c], d2[c], o.w, reach2);
              }
            }
          }
          if constexpr (FMT == FMT_CT16) {
            if (write_old) store16_w<NT>(b0 + q, wp);
            store16_w<NT>(b1 + q, wc);
            if (hp16) {
              const f16x8 lo = {(_Float16)U2[0].x, (_Float16)U2[0].y, (_Float16)U2[1].x, (_Float16)U2[1].y,
                                (_Float16)U2[2].x, (_Float16)U2[2].y, (_Float16)U2[3].x, (_Float16)U2[3].y};
              const f16x8 hi = {(_Float16)U2[NP - 4].x, (_Float16)U2[NP - 4].y, (_Float16)U2[NP - 3].x,
                                (_Float16)U2[NP - 3].y, (_Float16)U2[NP - 2].x, (_Float16)U2[NP - 2].y,
                                (_Float16)U2[NP - 1].x, (_Float16)U2[NP - 1].y};
              if (NT) {
                __builtin_nontemporal_store(lo, reinterpret_cast<f16x8*>(hp16 + q));
                __builtin_nontemporal_store(hi, reinterpret_cast<f16x8*>(hp16 + q + 8));
              } else {
                *reinterpret_cast<f16x8*>(hp16 + q) = lo;
                *reinterpret_cast<f16x8*>(hp16 + q + 8) = hi;
              }
            }
            if (FLOW) {
              store8_h<NT>(h0 + q, fx);
              store8_h<NT>(h0 + q + 8, fx + 8 % CPL);
              store8_h<NT>(h0 + G2 + q, fy);
              store8_h<NT>(h0 + G2 + q + 8, fy + 8 % CPL);
            }
          } else if constexpr (FMT == FMT_CT8) {
            const u32x2 fw = {wc[0], wc[NW - 1]}, pw = {wp[0], wp[NW - 1]};
            if (NT) {
              if (write_old) __builtin_nontemporal_store(pw, reinterpret_cast<u32x2*>(b0 + q));
              __builtin_nontemporal_store(fw, reinterpret_cast<u32x2*>(b1 + q));
            } else {
              if (write_old) *reinterpret_cast<u32x2*>(b0 + q) = pw;
              *reinterpret_cast<u32x2*>(b1 + q) = fw;
            }
            if (hp16) {
              const f16x8 u8v = {(_Float16)U2[0].x, (_Float16)U2[0].y, (_Float16)U2[1 % NP].x, (_Float16)U2[1 % NP].y,
                                 (_Float16)U2[2 % NP].x, (_Float16)U2[2 % NP].y, (_Float16)U2[3 % NP].x,
                                 (_Float16)U2[3 % NP].y};
              if (NT) __builtin_nontemporal_store(u8v, reinterpret_cast<f16x8*>(hp16 + q));
              else *reinterpret_cast<f16x8*>(hp16 + q) = u8v;
            }
            if (FLOW) {
              store8_h<NT>(h0 + q, fx);
              store8_h<NT>(h0 + G2 + q, fy);
            }
          } else if constexpr (FMT == FMT_CT4) {
            if (NT) {
              if (write_old) __builtin_nontemporal_store(wp[0], reinterpret_cast<uint32_t*>(b0 + q));
              __builtin_nontemporal_store(wc[0], reinterpret_cast<uint32_t*>(b1 + q));
            } else {
              if (write_old) *reinterpret_cast<uint32_t*>(b0 + q) = wp[0];
              *reinterpret_cast<uint32_t*>(b1 + q) = wc[0];
            }
            if (hp16) store4_h<NT>(hp16 + q, U2[0].x, U2[0].y, U2[NP - 1].x, U2[NP - 1].y);
            if (FLOW) {
              store4_h<NT>(h0 + q, fx[0], fx[1 % CPL], fx[2 % CPL], fx[3 % CPL]);
              store4_h<NT>(h0 + G2 + q, fy[0], fy[1 % CPL], fy[2 % CPL], fy[3 % CPL]);
            }
          } else {
            // byte 0xFF -> 255.0f, 0 -> 0.0f: the reference layout's occ * 255 values
            if (write_old)
              store4<NT>(m0 + q, (float)(wp[0] & 0xFFu), (float)((wp[0] >> 8) & 0xFFu), (float)((wp[0] >> 16) & 0xFFu),
                         (float)(wp[0] >> 24));
            store4<NT>(m1 + q, (float)(wc[0] & 0xFFu), (float)((wc[0] >> 8) & 0xFFu), (float)((wc[0] >> 16) & 0xFFu),
                       (float)(wc[0] >> 24));
            if (pp) store4<NT>(pp + q, U2[0].x, U2[0].y, U2[NP - 1].x, U2[NP - 1].y);
            if (FLOW) {
              store4<NT>(f0 + q, fx[0], fx[1 % CPL], fx[2 % CPL], fx[3 % CPL]);
              store4<NT>(f0 + G2 + q, fy[0], fy[1 % CPL], fy[2 % CPL], fy[3 % CPL]);
            }
          }
        }
      }
      return;
    }
    for (int t = wave; t < ntiles; t += 4) {
      const int band = t / ncb;
      const int cb = t - band * ncb;
      const int i0 = row0 + band * R, j0 = cb * C;
      const int i = i0 + r, j = j0 + cl;
      task(i0, i0 + R - 1, j0, j0 + C - 1, i, j, i * G + j, true);
    }
  } else {
    for (int q0 = qbeg + wave * WC; q0 < qend; q0 += 4 * WC) {
      // ---- wave chunk [q0, qlast] (WC consecutive cells) -> ego bounding box ----
      const int qlast = min(q0 + WC - 1, G2 - 1);
      const int i0 = q0 / G;
      const int r0 = q0 - i0 * G;
      const int i1 = i0 + small_div(r0 + (qlast - q0), invG);
      int j0 = 0, j1 = G - 1;
      if (i0 == i1) { j0 = r0; j1 = r0 + (qlast - q0); }
      const int off = r0 + lane * CPL;
      const int q = q0 + lane * CPL;
      const int di = small_div(off, invG);
      task(i0, i1, j0, j1, i0 + di, off - di * G, q, q < qend);
    }
  }
}

template <bool NT, bool XCD, bool FLOW, int FMT>
__global__ __launch_bounds__(256, (FMT == FMT_CT8 && !FLOW ? FFMP_CT8_MIN_WAVES : 1)) void raster_kernel(ffmp_cfg_t cfg, int64_t n, int32_t bpe,
                                                     int32_t cells_per_block,
                                                     const float* __restrict__ record,
                                                     const uint8_t* __restrict__ mask,
                                                     float* __restrict__ state_m, int64_t sm_stride,
                                                     int64_t sm_frame, int32_t newest_only,
                                                     float* __restrict__ pot,
                                                     float* __restrict__ flow, int32_t tile_log2r) {
  __shared__ float4 s_cur[FFMP_MAX_OBST], s_prev[FFMP_MAX_OBST];
  __shared__ float2 s_vel[FLOW ? FFMP_MAX_OBST : 1];
  __shared__ float s_hdr[FFMP_REC_HDR];
  const int64_t lb = logical_block<XCD>();
  const int64_t e = lb / bpe;
  const int tile = (int)(lb - e * bpe);
  if (e >= n) return;
  if (mask && !mask[e]) return;
  raster_env<NT, FLOW, FMT>(cfg, e, tile, cells_per_block, record, state_m, sm_stride, sm_frame, newest_only, pot, flow,
                       tile_log2r, s_cur, s_prev, s_vel, s_hdr);
#ifdef FFMP_TRACE
  __syncthreads();
  FFMP_RAS_STAMP(2);
#endif
}

// The fused step: one block per env.  Wave 0 steps the env (env_group, 64 lanes: integrator,
// obstacles, lidar, collision / reward / done, auto-reset, record), then the block rasters the
// env's whole plane from the record it just wrote.  The env step's float64 work of one block
// overlaps the store streams of the other blocks on the CU, instead of running as its own
// launch before the raster (~4 % of a C3 step).
// Compact CT4 without flow planes: held to 7 waves per SIMD (72 VGPRs), the stand-alone CT4
// raster's occupancy, which the compact store streams need (profiles/r02_occupancy.txt); the env
// phase then keeps 20 B/lane of scratch, the same as the stand-alone env kernel.  Otherwise the
// env phase's registers (89) would leave the raster 5 waves per SIMD.
template <bool FLOW, int FMT>
constexpr int kFusedMinWaves = (FMT == FMT_CT4 && !FLOW) ? 7 : (FMT == FMT_CT8 && !FLOW) ? FFMP_CT8_MIN_WAVES : 1;

template <bool NT, bool XCD, bool FLOW, int FMT>
__global__ __launch_bounds__(256, (kFusedMinWaves<FLOW, FMT>)) void step_raster_kernel(ffmp_cfg_t cfg, int64_t n, int64_t env_offset,
                                                          const int64_t* __restrict__ action, ffmp_state_t st,
                                                          ffmp_obs_t ob, ffmp_out_t out, int64_t sm_stride,
                                                          int64_t sm_frame, int32_t newest_only,
                                                          int32_t tile_log2r) {
  __shared__ double s_ox[FFMP_MAX_OBST], s_oy[FFMP_MAX_OBST], s_or[FFMP_MAX_OBST], s_orr[FFMP_MAX_OBST];
  __shared__ float4 s_ecur[FFMP_MAX_OBST], s_eprev[FFMP_MAX_OBST];
  __shared__ float2 s_foot[FFMP_MAX_FOOT + 1];  // + the cells' extent
  __shared__ float2 s_vel[FLOW ? FFMP_MAX_OBST : 1];
  __shared__ float s_hdr[FFMP_REC_HDR];
  const int64_t e = logical_block<XCD>();
  if (e >= n) return;
  FFMP_RAS_STAMP(0);
  if (threadIdx.x < 64) {
    stage_footprint(cfg, s_foot);
    // (one beam at a time where the block is held to more than 4 waves per SIMD: the chunked
    // lidar's registers would spill there)
    env_group<kEnvMode_Step, 64, (kFusedMinWaves<FLOW, FMT> > 4 ? 1 : FFMP_BEAM_CHUNK)>(cfg, env_offset, action, 0, st, ob, out, e, (int)threadIdx.x, s_ox, s_oy, s_or,
                                 s_orr, s_ecur, s_eprev, s_foot, s_hdr, FLOW ? s_vel : nullptr);
  }
  // The record reaches the raster through LDS: env_group left its ego discs of both frames in
  // s_ecur / s_eprev and wrote the header (and velocities) to s_hdr / s_vel — the same words it
  // stored to st.record — so the raster starts without a round trip to HBM for them.
  __syncthreads();
  FFMP_RAS_STAMP(3);
  raster_env<NT, FLOW, FMT, true>(cfg, e, 0, cfg.grid * cfg.grid, st.record, ob.state_m, sm_stride, sm_frame, newest_only,
                       ob.potential, ob.flow, tile_log2r, s_ecur, s_eprev, s_vel, s_hdr);
#ifdef FFMP_TRACE
  __syncthreads();
  FFMP_RAS_STAMP(2);
#endif
}

// The skewed step (ffmp_step_skewed): ONE launch = the raster of step t (blocks env_blocks..) and the
// env step of step t + 1 (blocks 0..env_blocks-1, four 64-lane env waves each, dispatched first),
// which have no dependency on each other: the raster reads only step t's record (written by the
// previous launch) and the env step writes step t + 1's state and its record into the OTHER record
// buffer.  The env waves' float64 latency chains then run beside raster blocks' store streams
// instead of as a launch of their own before the raster.  Float32 frames without flow planes: the
// combined kernel keeps the stand-alone raster's occupancy (4 waves per SIMD: the env path's 116
// VGPRs vs the raster's 108; 4 blocks per CU of LDS).  The two paths share one LDS block.
template <int LPE>
struct SkewEnvLds {
  static constexpr int W = 4, DS = 64;
  double ox[W][DS], oy[W][DS], orr_[W][DS], orrr[W][DS];
  float4 ecur[W][DS], eprev[W][DS];
  float2 foot[W][FFMP_MAX_FOOT + 1];
  int pref[W][DS], lo[W][DS];
};
struct SkewRasterLds {
  float4 cur[FFMP_MAX_OBST], prev[FFMP_MAX_OBST];
  float2 vel[1];
  float hdr[FFMP_REC_HDR];
};

template <bool NT, bool XCD, int LPE>
__global__ __launch_bounds__(256) void skew_kernel(ffmp_cfg_t cfg, int64_t n, int64_t env_offset,
                                                   const int64_t* __restrict__ action, ffmp_state_t st, ffmp_obs_t ob,
                                                   ffmp_out_t out, int32_t env_chunks, int32_t chunk_s, int32_t bpe,
                                                   int32_t cells_per_block, const float* __restrict__ record_r,
                                                   int64_t sm_stride, int64_t sm_frame, int32_t newest_only,
                                                   int32_t tile_log2r) {
  constexpr int W = 4, EPW = 64 / LPE;
  constexpr size_t kEnvB = sizeof(SkewEnvLds<LPE>), kRasB = sizeof(SkewRasterLds);
  __shared__ __attribute__((aligned(16))) char smem[kEnvB > kRasB ? kEnvB : kRasB];
  extern __shared__ uint32_t s_keys[];  // trace_discs' per-env beam minima (env blocks)
  // Block layout: env_chunks chunks of [8 env blocks, 8 * chunk_s raster blocks], then the rest of the
  // raster: the env blocks are spread over the first part of the launch (not all dispatched first —
  // at C3 they would fill every block slot for two rounds with no store in flight), one per XCD per
  // chunk, so each raster block keeps the XCD (blockIdx % 8) of its raster index.
  const int64_t b = blockIdx.x, chunk = 8 * ((int64_t)chunk_s + 1);
  int64_t env_block = -1, rb;
  if (b < (int64_t)env_chunks * chunk) {
    const int64_t c = b / chunk, off = b - c * chunk;
    if (off < 8) env_block = c * 8 + off;
    rb = c * 8 * chunk_s + (off - 8);
  } else {
    rb = (int64_t)env_chunks * 8 * chunk_s + (b - (int64_t)env_chunks * chunk);
  }
  if (env_block >= 0) {
    SkewEnvLds<LPE>& L = *reinterpret_cast<SkewEnvLds<LPE>*>(smem);
    const int wv = threadIdx.x >> 6;
    const int grp = (threadIdx.x & 63) / LPE;
    const int64_t e = (env_block * W + wv) * EPW + grp;
    const int lane = threadIdx.x & (LPE - 1);
    stage_footprint(cfg, L.foot[wv]);
    if (e >= n) return;
    const int g0 = grp * LPE;
    env_group<kEnvMode_Step, LPE, FFMP_BEAM_CHUNK, true, 1>(
        cfg, env_offset, action, 0, st, ob, out, e, lane, L.ox[wv] + g0, L.oy[wv] + g0, L.orr_[wv] + g0,
        L.orrr[wv] + g0, L.ecur[wv] + g0, L.eprev[wv] + g0, L.foot[wv], nullptr, nullptr,
        s_keys + ((size_t)wv * EPW + grp) * cfg.n_beams, L.pref[wv] + g0, L.lo[wv] + g0);
    return;
  }
  SkewRasterLds& R = *reinterpret_cast<SkewRasterLds*>(smem);
  // the raster's blocks as if they were a launch of their own
  int64_t lb = rb;
  if (XCD) {
    const int64_t per = ((int64_t)gridDim.x - 8 * (int64_t)env_chunks) / 8;
    if (lb < per * 8) lb = (lb % 8) * per + lb / 8;
  }
  const int64_t e = lb / bpe;
  const int tile = (int)(lb - e * bpe);
  if (e >= n) return;
  raster_env<NT, false, FMT_F32>(cfg, e, tile, cells_per_block, record_r, ob.state_m, sm_stride, sm_frame, newest_only,
                                 ob.potential, nullptr, tile_log2r, R.cur, R.prev, R.vel, R.hdr);
}

// ============================================================================
// Legacy FFMP methods as batched kernels (one thread per env).
// ============================================================================
__global__ void reward_done_kernel(ffmp_cfg_t cfg, int64_t n, const double* __restrict__ scan,
                                   int32_t scan_len, const float* __restrict__ local_map,
                                   int64_t map_stride, const uint8_t* __restrict__ collide_in,
                                   const uint8_t* __restrict__ goal_in,
                                   const double* __restrict__ rel_goal,
                                   const uint8_t* __restrict__ is_first, double* d0, double* reward,
                                   uint8_t* done, uint8_t* is_goal, uint8_t* collide) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  bool col = collide_in ? (collide_in[e] != 0) : false;
  if (scan) {
    for (int l = 0; l < scan_len; ++l) {
      const double r = scan[e * scan_len + l];
      if (r != 0.0 && r < cfg.robot_r) { col = true; break; }
    }
  }
  if (local_map) {
    const float* m = local_map + e * map_stride;
    const int c = cfg.grid / 2;
    for (int f = 0; f < cfg.n_foot; ++f)
      if (m[(int64_t)(c + cfg.foot_di[f]) * cfg.grid + (c + cfg.foot_dj[f])] > 0.0f) { col = true; break; }
  }
  const double dist = rel_goal[e * 2];
  const bool goal = goal_in ? (goal_in[e] != 0) : (dist < cfg.goal_thr);
  if (is_first[e]) d0[e] = dist;
  reward[e] = reward_calc(dist, d0[e], col, goal);
  done[e] = col || goal;
  is_goal[e] = goal;
  collide[e] = col;
}

// One env's reward / done with its inputs in the kernel's arguments (ffmp_reward_done_packed flag 8):
// no host -> device copy; the outputs go straight into the caller's pinned block through its device
// view.  The same operations as reward_done_kernel for n = 1 without a local map.
struct PackedArgs {
  double scan[FFMP_PACKED_ARG_BEAMS];
  double dist, d0, robot_r, goal_thr;
  int32_t scan_len;
  uint8_t is_first, collide_in, goal_in, flags;
};
__global__ void reward_done_args_kernel(PackedArgs a, uint8_t* __restrict__ out) {
  // the beams over the wave's 64 lanes: "some beam hits" does not depend on the order it is tested in
  bool hit = false;
  for (int l = (int)threadIdx.x; l < a.scan_len; l += 64) {
    const double r = a.scan[l];
    hit = hit || (r != 0.0 && r < a.robot_r);
  }
  const bool any_hit = __ballot(hit) != 0ull;
  if (threadIdx.x != 0) return;
  const bool col = ((a.flags & 1) ? (a.collide_in != 0) : false) || any_hit;
  const bool goal = (a.flags & 2) ? (a.goal_in != 0) : (a.dist < a.goal_thr);
  const double d0 = a.is_first ? a.dist : a.d0;
  *reinterpret_cast<double*>(out) = reward_calc(a.dist, d0, col, goal);
  *reinterpret_cast<double*>(out + 8) = d0;
  out[16] = col || goal;
  out[17] = goal;
  out[18] = col;
}

__global__ void footprint_kernel(ffmp_cfg_t cfg, int64_t n, const float* __restrict__ local_map,
                                 int64_t map_stride, uint8_t* collide) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const float* m = local_map + e * map_stride;
  const int c = cfg.grid / 2;
  bool col = false;
  for (int f = 0; f < cfg.n_foot; ++f)
    col |= m[(int64_t)(c + cfg.foot_di[f]) * cfg.grid + (c + cfg.foot_dj[f])] > 0.0f;
  collide[e] = col;
}

template <typename T>
__global__ __launch_bounds__(256) void scan_kernel(int64_t n, int32_t L, const T* __restrict__ ranges,
                                                   double thr, uint8_t* collide, T* min_r) {
  const int64_t e = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (e >= n) return;
  bool col = false;
  T mn = (T)__builtin_inf();
  for (int l = lane; l < L; l += 64) {
    const T r = ranges[e * L + l];
    if (r != (T)0) {
      col |= (double)r < thr;
      mn = r < mn ? r : mn;  // NaN never replaces
    }
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    const T o = __shfl_xor(mn, off);
    mn = o < mn ? o : mn;
  }
  col = __any(col);
  if (lane == 0) {
    collide[e] = col;
    if (min_r) min_r[e] = mn;
  }
}

template <typename T>
int scan_impl(int64_t n, int32_t L, const T* ranges, double thr, uint8_t* collide, T* min_r,
                     void* stream) {
  if (n < 0 || L < 0) return fail(FFMP_E_ARG, "negative n or L");
  if ((L > 0 && !ranges) || !collide) return fail(FFMP_E_ARG, "ranges/collide is NULL");
  if (n == 0) return FFMP_OK;
  hipLaunchKernelGGL(scan_kernel<T>, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, n, L,
                     ranges, thr, collide, min_r);
  return check_launch("ffmp_scan_collision");
}


// ============================================================================
// Episode bookkeeping (src/train.py:501-505, 579-587, 593, 607, 611-682), one thread per env.
// Counts for totals[] are wave ballots: one atomic per counter per wave.
// ============================================================================
// ============================================================================
// Exhaustive check of the raster's sqrt_rn / rcp_rn against the IEEE sqrtf and 1.0f / d over the
// float bit patterns [lo, hi) (grid-stride; one global atomic per mismatching wave).
// ============================================================================
__global__ __launch_bounds__(256) void exact_math_kernel(int32_t which, uint32_t lo, uint32_t hi,
                                                          unsigned long long* mismatches, uint32_t* first_bits) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t b = (uint64_t)lo + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; b < hi; b += stride) {
    const float x = __uint_as_float((uint32_t)b);
    const float fast = which == 0 ? sqrt_rn(x) : rcp_rn(x);
    const float ieee = which == 0 ? sqrtf(x) : 1.0f / x;
    const bool bad = __float_as_uint(fast) != __float_as_uint(ieee);
    const unsigned long long m = __ballot(bad);
    if (bad && (int)(threadIdx.x & 63) == __builtin_ctzll(m)) atomicMin(first_bits, (uint32_t)b);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd(mismatches, (unsigned long long)__popcll(m));
  }
}

__device__ __forceinline__ void wave_count(uint64_t* totals, int k, bool pred) {
  const unsigned long long m = __ballot(pred);
  if ((threadIdx.x & 63) == 0 && m) atomicAdd((unsigned long long*)&totals[k], (unsigned long long)__popcll(m));
}

__global__ __launch_bounds__(256) void episode_init_kernel(int64_t n, const uint8_t* __restrict__ mask,
                                                           int32_t flags, ffmp_episode_t ep) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = e < n && !(mask && !mask[e]);
  const bool it0 = (flags & FFMP_EP_RESET_ITER) != 0;  // one (no-goal, not-done) iteration
  if (act) {
    ep.reach_bits[e] = 0;
    ep.reach_len[e] = it0 ? 1 : 0;
    ep.reach_rate[e] = 0.0;
    ep.step[e] = it0 ? 1 : 0;
    ep.episode[e] = 0;
    ep.total_step[e] = it0 ? 1 : 0;
    ep.is_first[e] = it0 ? 0 : 1;
    ep.complete[e] = 0;
  }
  if (ep.totals) wave_count(ep.totals, 6, act && it0);
}

__global__ __launch_bounds__(256) void episode_update_kernel(int64_t n, ffmp_out_t out, int32_t window,
                                                             int32_t max_steps, double threshold, int32_t flags,
                                                             ffmp_episode_t ep) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool act = e < n;
  const bool it0 = (flags & FFMP_EP_RESET_ITER) != 0;
  bool goal = false, done = false, trunc = false, col = false, fin = false;
  if (act) {
    goal = out.is_goal[e] != 0;
    col = out.collide[e] != 0;
    const int32_t step = ep.step[e];
    // :579-587  reach_times.append(is_goal); keep the last REACH_MEMORY_CAPACITY; np.average
    const uint64_t keep = window >= 64 ? ~0ull : ((1ull << window) - 1ull);
    uint64_t bits = ((ep.reach_bits[e] << 1) | (goal ? 1ull : 0ull)) & keep;
    int32_t len = min(ep.reach_len[e] + 1, window);
    double rate = (double)__popcll(bits) / (double)len;
    // :607  if step == MAX_STEPS: is_done = True
    const bool own_trunc = max_steps > 0 && step == max_steps;
    done = (out.done[e] != 0) || own_trunc;
    trunc = done && ((out.truncated[e] != 0) || (own_trunc && !out.done[e]));
    if (done) {  // :611-663
      ep.episode[e] += 1;
      fin = (flags & FFMP_EP_ARMED) && rate > threshold;  // :644
      if (fin) ep.complete[e] = 1;
      if (it0) {  // the next episode's reset-observation iteration: no goal, not done
        bits = (bits << 1) & keep;
        len = min(len + 1, window);
        rate = (double)__popcll(bits) / (double)len;
        ep.step[e] = 1;
        ep.total_step[e] += 1;
        ep.is_first[e] = 0;
      } else {
        ep.step[e] = 0;
        ep.is_first[e] = 1;
      }
    } else {  // :593, :681-682
      ep.step[e] = step + 1;
      ep.total_step[e] += 1;
      ep.is_first[e] = 0;
    }
    ep.reach_bits[e] = bits;
    ep.reach_len[e] = len;
    ep.reach_rate[e] = rate;
  }
  if (ep.totals) {
    wave_count(ep.totals, 0, act);
    wave_count(ep.totals, 1, done);
    wave_count(ep.totals, 2, goal);
    wave_count(ep.totals, 3, col);
    wave_count(ep.totals, 4, trunc);
    wave_count(ep.totals, 5, fin);
    wave_count(ep.totals, 6, act && (!done || it0));
  }
}

static int check_episode(const ffmp_episode_t* ep) {
  if (!ep || !ep->reach_bits || !ep->reach_len || !ep->reach_rate || !ep->step || !ep->episode ||
      !ep->total_step || !ep->is_first || !ep->complete)
    return fail(FFMP_E_ARG, "episode struct or one of its arrays is NULL");
  return FFMP_OK;
}

// LDS a block may use on this device (static + dynamic), read once
size_t device_lds_limit() {
  static const size_t lim = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&v, hipDeviceAttributeMaxSharedMemoryPerBlock, dev) != hipSuccess || v <= 0)
      return (size_t)64 * 1024;
    return (size_t)v;
  }();
  return lim;
}

// false (nothing launched) when the block's LDS — the static disc / footprint arrays, which grow
// with the discs per lane, plus trace_discs' dynamic beam minima (W x envs per wave x L words) —
// exceeds what a block may use: the caller then tries a layout that needs less
template <int MODE, int W, int LPE, int DPL>
bool launch_env_t(const ffmp_cfg_t& cfg, int64_t n, int64_t env_offset, const int64_t* action, const uint8_t* mask,
                  int32_t initial, const ffmp_state_t& st, const ffmp_obs_t& ob, const ffmp_out_t& o,
                  hipStream_t s) {
  static const size_t static_lds = [] {
    hipFuncAttributes a{};
    return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&env_kernel<MODE, W, LPE, DPL>)) == hipSuccess
               ? (size_t)a.sharedSizeBytes
               : (size_t)0;
  }();
  const int64_t per_block = (int64_t)W * (64 / LPE);
  const unsigned blocks = (unsigned)((n + per_block - 1) / per_block);
  const size_t lds = (size_t)W * (64 / LPE) * (size_t)cfg.n_beams * sizeof(uint32_t);  // trace_discs' beam minima
  if (static_lds + lds > device_lds_limit()) return false;
  hipLaunchKernelGGL((env_kernel<MODE, W, LPE, DPL>), dim3(blocks), dim3(64 * W), lds, s, cfg, n, env_offset, action,
                     mask, initial, st, ob, o);
  return true;
}

// (lanes per env, discs per lane) pairs with an env_kernel instance; false if there is none or its
// block would not fit the LDS
template <int MODE, int W>
bool launch_env_mode(int lpe, int dpl, const ffmp_cfg_t& cfg, int64_t n, int64_t env_offset, const int64_t* action,
                     const uint8_t* mask, int32_t initial, const ffmp_state_t& st, const ffmp_obs_t& ob,
                     const ffmp_out_t& o, hipStream_t s) {
#define FFMP_ENV_CASE(L_, D_)                                                                    \
  if (lpe == L_ && dpl == D_) return launch_env_t<MODE, W, L_, D_>(cfg, n, env_offset, action, mask, initial, st, ob, o, s);
  FFMP_ENV_CASE(16, 1) FFMP_ENV_CASE(32, 1) FFMP_ENV_CASE(64, 1) FFMP_ENV_CASE(8, 2) FFMP_ENV_CASE(16, 2)
  FFMP_ENV_CASE(4, 4) FFMP_ENV_CASE(8, 1)
#undef FFMP_ENV_CASE
  return false;
}

template <int W>
bool launch_env_lpe(int mode, int lpe, int dpl, const ffmp_cfg_t& cfg, int64_t n, int64_t env_offset,
                    const int64_t* action, const uint8_t* mask, int32_t initial, const ffmp_state_t& st,
                    const ffmp_obs_t& ob, const ffmp_out_t& o, hipStream_t s) {
  if (mode == kEnvMode_Step)
    return launch_env_mode<kEnvMode_Step, W>(lpe, dpl, cfg, n, env_offset, action, mask, initial, st, ob, o, s);
  return launch_env_mode<kEnvMode_Reset, W>(lpe, dpl, cfg, n, env_offset, action, mask, initial, st, ob, o, s);
}

// ============================================================================
// make_temporal_maps over k frames (ffmp_temporal_maps, src/train.py:474-486): out[e][c] is the
// frame of lag d = k-1-c, clamped to the episode start (min(d, since[e]): on is_first the
// reference refills map_memory with the first frame).  A pure HBM copy, k planes read and
// written per env: a block moves 16 KiB of one output plane, 16-B loads and stores.
// ============================================================================
struct LagOffsets {
  int64_t b[FFMP_MAX_SERIES];  // byte offset of lag d's frame of env 0 from `frames`
};

typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void temporal_maps_kernel(const char* __restrict__ frames, LagOffsets lag,
                                                            int32_t k, int64_t env_b, int64_t plane_b,
                                                            const int32_t* __restrict__ since, int32_t chunks,
                                                            char* __restrict__ out) {
  const int64_t pc = blockIdx.x / chunks;  // output plane (e, c)
  const int chunk = (int)(blockIdx.x - pc * chunks);
  const int64_t e = pc / k;
  const int c = (int)(pc - e * k);
  int d = k - 1 - c;
  if (since) d = min(d, max(since[e], 0));
  d = __builtin_amdgcn_readfirstlane(d);  // block-uniform: the offset comes from the kernel arguments
  const u32x4_t* src = reinterpret_cast<const u32x4_t*>(frames + lag.b[d] + e * env_b);
  u32x4_t* dst = reinterpret_cast<u32x4_t*>(out + pc * plane_b);
  const int64_t n16 = plane_b / 16;
  const int64_t i0 = (int64_t)chunk * 1024 + threadIdx.x;
  u32x4_t v[4];
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (i0 + 256 * u < n16) v[u] = __builtin_nontemporal_load(src + i0 + 256 * u);
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (i0 + 256 * u < n16) dst[i0 + 256 * u] = v[u];
}

// ============================================================================
// The 4-channel BEV image of the reference's 12-channel option (src/train.py:66 "(occupancy(MONO)
// + flow(RGB)) * series(3 steps)", gym_ffmp/envs/ffmp.py:16): [occupancy, R, G, B] per cell, the
// occupancy of the newest frame as stored and the motion flow (cfg.flow: the covering disc's ego
// velocity) as colour.  The reference's RGB came from BEV nodes outside its repository, so the
// encoding is stated here (include/ffmp.h ffmp_bev_image), float32 operations in this order:
//   R = clamp(rint(127.5 + 127.5 * (vx / vmax)), 0, 255), G the same of vy,
//   B = clamp(rint(255 * (sqrt(vx*vx + vy*vy) / vmax)), 0, 255).
// Elementwise and HBM-bound (3 planes read, 4 written per env); a thread does 4 consecutive
// cells when the plane allows it (G even), else 1.
// ============================================================================
FFMP_DEV float flow_axis_rgb(float v, float vmax) {
  const float q = v / vmax;
  const float a = 127.5f * q;
  return fminf(fmaxf(rintf(127.5f + a), 0.0f), 255.0f);
}

FFMP_DEV float flow_speed_rgb(float vx, float vy, float vmax) {
  const float s = sqrtf(vx * vx + vy * vy);
  const float q = s / vmax;
  return fminf(fmaxf(rintf(255.0f * q), 0.0f), 255.0f);
}

template <bool CT, int V>
__global__ __launch_bounds__(256) void bev_image_kernel(int64_t n, const void* __restrict__ occ, int64_t occ_env,
                                                        const void* __restrict__ flow, int64_t plane, int32_t chunks,
                                                        float vmax, void* __restrict__ out, int64_t out_env) {
  const int64_t e = blockIdx.x / chunks;
  const int64_t q0 = ((int64_t)(blockIdx.x - e * chunks) * 256 + threadIdx.x) * V;
  if (e >= n || q0 >= plane) return;
  float o[V], fx[V], fy[V];
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const int64_t q = q0 + u;
    if (CT) {
      o[u] = (float)static_cast<const uint8_t*>(occ)[e * occ_env + q];
      fx[u] = (float)static_cast<const _Float16*>(flow)[e * 2 * plane + q];
      fy[u] = (float)static_cast<const _Float16*>(flow)[e * 2 * plane + plane + q];
    } else {
      o[u] = static_cast<const float*>(occ)[e * occ_env + q];
      fx[u] = static_cast<const float*>(flow)[e * 2 * plane + q];
      fy[u] = static_cast<const float*>(flow)[e * 2 * plane + plane + q];
    }
  }
#pragma unroll
  for (int u = 0; u < V; ++u) {
    const float c[4] = {o[u], flow_axis_rgb(fx[u], vmax), flow_axis_rgb(fy[u], vmax), flow_speed_rgb(fx[u], fy[u], vmax)};
#pragma unroll
    for (int ch = 0; ch < 4; ++ch) {
      const int64_t at = e * out_env + ch * plane + q0 + u;
      if (CT) static_cast<uint8_t*>(out)[at] = (uint8_t)c[ch];
      else static_cast<float*>(out)[at] = c[ch];
    }
  }
}

// ============================================================================
// C ABI
// ============================================================================
namespace {

// log2 of the rows of a 2-D wave tile (FFMP_RASTER_TILE*), 0 = 1-D chunks
int32_t tile_rows_log2(int32_t flags) {
  return (flags & FFMP_RASTER_TILE16) ? 4 : (flags & FFMP_RASTER_TILE8) ? 3 : (flags & FFMP_RASTER_TILE4) ? 2
       : (flags & FFMP_RASTER_TILE2) ? 1 : 0;
}

// The raster instantiation for an obs format: compact planes use 16 cells per lane when every
// lane's 16 cells stay in one row (G % 16 == 0) unless FFMP_RASTER_NARROW asks for 4.
int raster_format(bool compact, int grid, int32_t flags) {
  if (!compact) return FMT_F32;
  if (flags & FFMP_RASTER_NARROW) return FMT_CT4;
  if ((flags & FFMP_RASTER_MID8) && grid % 8 == 0) return FMT_CT8;
  return grid % 16 == 0 ? FMT_CT16 : FMT_CT4;
}

// The scripted reactive controller of ffmp_policy_reactive: one thread per env reads the env's
// relative goal and a short ray of cells ahead of the robot on its newest frame (row index = ego
// x = heading, ffmp_device.h cell_coord), and picks the action id 7 * vi + wi (config.py:25-58).
template <typename T>
__global__ __launch_bounds__(256) void policy_reactive_kernel(int64_t n, int32_t grid, const T* __restrict__ newest,
                                                              int64_t env_stride, const float* __restrict__ state_g,
                                                              int32_t look0, int32_t look1, float slow_dist,
                                                              int64_t* __restrict__ action) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const float2 g = reinterpret_cast<const float2*>(state_g)[e];
  int wi = (int)rintf(g.y / 0.2f) + 3;  // turn towards the goal (orient > 0: to the left, w > 0)
  wi = wi < 0 ? 0 : wi > 6 ? 6 : wi;
  const T* f = newest + e * env_stride + (int64_t)(grid / 2) * grid + grid / 2;
  bool blocked = false;
  for (int d = look0; d <= look1; ++d) blocked |= f[(int64_t)d * grid] > (T)0;
  int vi = g.x < slow_dist ? 1 : 3;
  if (blocked) {
    vi = 0;
    if (wi == 3) wi = 6;  // obstacle straight ahead and the goal too: turn on the spot (left)
  }
  action[e] = 7 * vi + wi;
}

// Calls f(NT, XCD, FLOW, FMT) with std::integral_constant arguments for the runtime choice (the
// compact formats' flow planes are binary16).
template <class F>
void dispatch_variant(int fmt, bool nt, bool xcd, bool fl, F&& f) {
  using T = std::true_type;
  using N = std::false_type;
  auto with_fmt = [&](auto NT_, auto XCD_) {
    if (fmt == FMT_CT16) {
      if (fl) f(NT_, XCD_, T{}, std::integral_constant<int, FMT_CT16>{});
      else f(NT_, XCD_, N{}, std::integral_constant<int, FMT_CT16>{});
    } else if (fmt == FMT_CT8) {
      if (fl) f(NT_, XCD_, T{}, std::integral_constant<int, FMT_CT8>{});
      else f(NT_, XCD_, N{}, std::integral_constant<int, FMT_CT8>{});
    } else if (fmt == FMT_CT4) {
      if (fl) f(NT_, XCD_, T{}, std::integral_constant<int, FMT_CT4>{});
      else f(NT_, XCD_, N{}, std::integral_constant<int, FMT_CT4>{});
    }
    else if (fl) f(NT_, XCD_, T{}, std::integral_constant<int, FMT_F32>{});
    else f(NT_, XCD_, N{}, std::integral_constant<int, FMT_F32>{});
  };
  if (nt) {
    if (xcd) with_fmt(T{}, T{});
    else with_fmt(T{}, N{});
  } else {
    if (xcd) with_fmt(N{}, T{});
    else with_fmt(N{}, N{});
  }
}

}  // namespace

extern "C" {

int ffmp_abi_version(void) { return FFMP_ABI_VERSION; }

int32_t ffmp_set_tuning(int32_t key, int32_t value) {
  Tuning& t = tuning();
  int32_t prev;
  switch (key) {
    case FFMP_TUNE_RASTER_CPB:
      if (value != 0 && (value < 1024 || value % 1024 != 0)) return fail(FFMP_E_ARG, "cells per block must be a multiple of 1024");
      prev = t.cells_per_block;
      t.cells_per_block = value ? value : 4096;
      return prev;
    case FFMP_TUNE_RASTER_NT:
      if (value < 0 || value > 2) return fail(FFMP_E_ARG, "store flavour must be 0 (auto), 1 (plain) or 2 (nt)");
      prev = t.nontemporal + 1;
      t.nontemporal = value - 1;
      return prev;
    case FFMP_TUNE_RASTER_XCD:
      prev = t.xcd_remap;
      t.xcd_remap = value != 0;
      return prev;
    case FFMP_TUNE_ENV_WAVES:
      if (value != 1 && value != 4) return fail(FFMP_E_ARG, "env waves must be 1 or 4");
      prev = t.env_waves;
      t.env_waves = value;
      return prev;
    case FFMP_TUNE_ENV_LANES:
      if (value != 0 && value != 4 && value != 8 && value != 16 && value != 32 && value != 64)
        return fail(FFMP_E_ARG, "env lanes must be 0 (auto), 4, 8, 16, 32 or 64");
      prev = t.env_lanes;
      t.env_lanes = value;
      return prev;
    case FFMP_TUNE_CONV_MFMA:
      if (value != 0 && value != 16 && value != 32)
        return fail(FFMP_E_ARG, "conv MFMA shape must be 0 (each kernel's best), 16 (16x16x32) or 32 (32x32x16)");
      return ffmp_detail::conv_mfma_swap(value);
    case FFMP_TUNE_CONV_KYS:
      if (value != 0 && value != 1 && value != 2 && value != 4)
        return fail(FFMP_E_ARG, "conv kernel rows per ring step must be 0 (by shape), 1, 2 or 4");
      return ffmp_detail::conv_kys_swap(value);
    case FFMP_TUNE_CONV_LB:
      if (value != 0 && value != 1) return fail(FFMP_E_ARG, "conv B-through-LDS must be 0 or 1");
      return ffmp_detail::conv_lb_swap(value);
    case FFMP_TUNE_CONV_WGPF:
      if (value != 0 && value != 1) return fail(FFMP_E_ARG, "weight-gradient prefetch must be 0 or 1");
      return ffmp_detail::conv_wgpf_swap(value);
    case FFMP_TUNE_CONV_WGDMA:
      if (value < 0 || value > 4) return fail(FFMP_E_ARG, "conv weight-gradient DMA must be 0-4");
      return ffmp_detail::conv_wgdma_swap(value);
    case FFMP_TUNE_CONV_PIN:
      if (value != 0 && value != 1) return fail(FFMP_E_ARG, "conv pinned schedule must be 0 or 1");
      return ffmp_detail::conv_pin_swap(value);
    case FFMP_TUNE_CONV_PLANAR:
      if (value != 0 && value != 1) return fail(FFMP_E_ARG, "conv planar slots must be 0 or 1");
      return ffmp_detail::conv_planar_swap(value);
    case FFMP_TUNE_CONV_MBW:
      if (value < 0 || value > 4) return fail(FFMP_E_ARG, "conv blocks per wave must be 0-4");
      return ffmp_detail::conv_mbw_swap(value);
    case FFMP_TUNE_CONV_BA2:
      if (value < 0 || value > 2) return fail(FFMP_E_ARG, "conv pinned-schedule variant must be 0-2");
      return ffmp_detail::conv_ba2_swap(value);
    case FFMP_TUNE_RING_EXTRA:
      if (value < 0) return fail(FFMP_E_ARG, "ring extra pieces: 0 (default) or 1 + the cap");
      return ffmp_detail::ring_extra_swap(value);
    default:
      return fail(FFMP_E_ARG, "unknown tuning key %d", key);
  }
}
const char* ffmp_last_error(void) { return g_err; }

int64_t ffmp_layout(int32_t which) {
  switch (which) {
    case 0: return (int64_t)sizeof(ffmp_cfg_t);
    case 1: return (int64_t)sizeof(ffmp_state_t);
    case 2: return (int64_t)sizeof(ffmp_obs_t);
    case 3: return (int64_t)sizeof(ffmp_out_t);
    case 4: return (int64_t)offsetof(ffmp_cfg_t, res);
    case 5: return (int64_t)offsetof(ffmp_cfg_t, res_f);
    case 6: return (int64_t)offsetof(ffmp_cfg_t, seed);
    case 7: return (int64_t)offsetof(ffmp_cfg_t, beam_cs);
    case 8: return (int64_t)sizeof(ffmp_episode_t);
    case 9: return (int64_t)offsetof(ffmp_obs_t, format);
    default: return -1;
  }
}

int ffmp_footprint(int32_t grid, double res, double robot_r, int32_t* di, int32_t* dj, int32_t cap) {
  if (grid <= 0 || !(res > 0.0)) return fail(FFMP_E_ARG, "bad grid/res");
  // ffmp.py:87-94 with map_range = grid * res: cells whose corner-index
  // position lies within robot_r of the map centre.  Only a window around the
  // centre can qualify; scanning it in (i, j) order reproduces the list order.
  const double map_range = (double)grid * res;
  const int w = (int)ceil(robot_r / res) + 2;
  const int c = grid / 2;
  int cnt = 0;
  for (int i = c - w; i <= c + w; ++i) {
    if (i < 0 || i >= grid) continue;
    for (int j = c - w; j <= c + w; ++j) {
      if (j < 0 || j >= grid) continue;
      const double xp = pow(i * res - 0.5 * map_range, 2.0);
      const double yp = pow(j * res - 0.5 * map_range, 2.0);
      if (sqrt(xp + yp) <= robot_r) {
        if (cnt < cap && di && dj) { di[cnt] = i - c; dj[cnt] = j - c; }
        ++cnt;
      }
    }
  }
  return cnt;
}

static int launch_env(int mode, const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset,
                      const int64_t* action, const uint8_t* mask, int32_t initial,
                      ffmp_state_t* state, ffmp_obs_t* obs, ffmp_out_t* out, void* stream) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (n < 0 || env_offset < 0) return fail(FFMP_E_ARG, "negative n or env_offset");
  if (!state || !obs) return fail(FFMP_E_ARG, "state/obs is NULL");
  if (!state->pose || !state->goal || !state->d0 || !state->t || !state->episode || !state->record || !state->err)
    return fail(FFMP_E_ARG, "a state pointer is NULL");
  if (cfg->n_obst > 0 && (!state->obst || !state->obst_r)) return fail(FFMP_E_ARG, "obstacle state NULL");
  if (!obs->state_g || !obs->state_v || !obs->state_t || !obs->grad)
    return fail(FFMP_E_ARG, "an obs pointer is NULL");
  if (cfg->n_beams > 0 && !obs->lidar) return fail(FFMP_E_ARG, "obs.lidar NULL with n_beams > 0");
  if (mode == kEnvMode_Step) {
    if (!action) return fail(FFMP_E_ARG, "action is NULL");
    if (!out || !out->reward || !out->done || !out->is_goal || !out->collide || !out->truncated)
      return fail(FFMP_E_ARG, "an out pointer is NULL");
  }
  if (n == 0) return FFMP_OK;
  if (n > 0x7fffffffLL / 64) return fail(FFMP_E_ARG, "n too large for one launch: %lld", (long long)n);  // <= 64 lanes per env
  ffmp_out_t o = out ? *out : ffmp_out_t{};
  const Tuning& tu = tuning();
  // lanes per env: the fewest that hold the discs (lane k holds disc k).  Round 1 gave many-beam
  // configs more lanes to keep the one-beam-at-a-time lidar loop short; with three beams per chunk
  // the per-env scalar work dominates and fewer, longer beam loops win: C3 (K = 16, L = 180) 79 us
  // at 32 lanes -> 68 at 16, the C5 share (K = 32, L = 360) 83 at 64 -> 77 at 32
  // (profiles/r03c_beam_chunk.txt).
  // Round 4: a lane may hold several discs (k = lane + j * lanes, j < discs per lane), so that more
  // envs share a wave: FFMP_TUNE_ENV_LANES picks the lanes per env and the discs per lane follow
  // (ceil(K / lanes)); a pair without a kernel instance falls back to one disc per lane.  Measured
  // (profiles/r04k_env_lanes.txt): two discs per lane at 8 lanes is slower at C3 (52.5 vs 43.7 us:
  // the lidar's (disc, beam) pairs are shared by half the lanes; the rest takes the same 30 us), so
  // the default stays one disc per lane, the fewest lanes that hold them — 8 for K <= 8 (C2 12.1 vs
  // 12.6 us at 16).
  const int need = cfg->n_obst <= 8 ? 8 : cfg->n_obst <= 16 ? 16 : cfg->n_obst <= 32 ? 32 : 64;
  int lpe = tu.env_lanes ? tu.env_lanes : need;
  int dpl = cfg->n_obst <= lpe ? 1 : (cfg->n_obst + lpe - 1) / lpe;
  const hipStream_t hs = (hipStream_t)stream;
  const bool w4 = tu.env_waves == 4;
  auto try_launch = [&](bool four, int l, int d) {
    return four ? launch_env_lpe<4>(mode, l, d, *cfg, n, env_offset, action, mask, initial, *state, *obs, o, hs)
                : launch_env_lpe<1>(mode, l, d, *cfg, n, env_offset, action, mask, initial, *state, *obs, o, hs);
  };
  // the tuned layout; one wave per block (a quarter of the LDS); one disc per lane on the fewest
  // lanes that hold the discs (the smallest static arrays) — the last always fits (64 lanes x 1
  // disc x 72 B + one env's L <= 1024 words)
  const bool ok = try_launch(w4, lpe, dpl) || (w4 && try_launch(false, lpe, dpl)) ||
                  (w4 && try_launch(true, need, 1)) || try_launch(false, need, 1);
  if (!ok)
    return fail(FFMP_E_ARG, "no env_kernel layout fits the %zu B of LDS a block may use (K = %d, L = %d)",
                device_lds_limit(), cfg->n_obst, cfg->n_beams);
  return check_launch(mode == kEnvMode_Step ? "ffmp_step_state" : "ffmp_reset");
}

int ffmp_reset(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset, const uint8_t* mask,
               int32_t initial, ffmp_state_t* state, ffmp_obs_t* obs, void* stream) {
  return launch_env(kEnvMode_Reset, cfg, n, env_offset, nullptr, mask, initial, state, obs, nullptr, stream);
}

int ffmp_step_state(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset, const int64_t* action,
                    ffmp_state_t* state, ffmp_obs_t* obs, ffmp_out_t* out, void* stream) {
  return launch_env(kEnvMode_Step, cfg, n, env_offset, action, nullptr, 0, state, obs, out, stream);
}

int ffmp_raster_ex(const ffmp_cfg_t* cfg, int64_t n, const float* record, const uint8_t* mask,
                   ffmp_obs_t* obs, int32_t cells_per_block, int32_t flags, void* stream) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (n < 0) return fail(FFMP_E_ARG, "negative n");
  if (!record || !obs || !obs->state_m) return fail(FFMP_E_ARG, "record/obs/state_m is NULL");
  if (cells_per_block != 0 && (cells_per_block < 1024 || cells_per_block % 1024 != 0))
    return fail(FFMP_E_ARG, "cells_per_block must be 0 or a multiple of 1024, got %d", cells_per_block);
  if ((flags & FFMP_RASTER_NT) && (flags & FFMP_RASTER_PLAIN)) return fail(FFMP_E_ARG, "NT and PLAIN both set");
  if (int rc2 = check_format(obs, cfg->flow != 0)) return rc2;
  if (n == 0) return FFMP_OK;
  const int G2 = cfg->grid * cfg->grid;
  const int cpb_max = cells_per_block ? cells_per_block : 4096;
  const int cpb = G2 < cpb_max ? ((G2 + 1023) / 1024) * 1024 : cpb_max;
  const int bpe = (G2 + cpb - 1) / cpb;
  // a launch holds at most 2^31 - 1 work-items: larger batches go out as several launches over
  // consecutive env ranges (the whole C5 workload in the compact format is 131,072 x 64 blocks)
  const int64_t max_envs = (0x7fffffffLL / 256) / bpe;
  if (max_envs < 1) return fail(FFMP_E_ARG, "a raster plane needs too many blocks: %d", bpe);
  const bool nt = (flags & FFMP_RASTER_NT) ? true : (flags & FFMP_RASTER_PLAIN) ? false : (G2 <= 16384);
  const bool xcd = (flags & FFMP_RASTER_XCD) != 0;
  const bool fl = cfg->flow != 0;
  if (fl && !obs->flow) return fail(FFMP_E_ARG, "cfg.flow is set but obs.flow is NULL");
  const bool ct = obs->format == FFMP_OBS_U8F16;
  const int64_t sm_stride = obs->state_m_stride ? obs->state_m_stride : 2 * (int64_t)G2;
  const int64_t sm_frame = obs->state_m_frame_stride ? obs->state_m_frame_stride : (int64_t)G2;
  const int64_t sm_frame_abs = sm_frame < 0 ? -sm_frame : sm_frame;  // negative: newest in a lower slot
  if (sm_stride < (int64_t)G2 || sm_frame_abs < (int64_t)G2 ||
      (sm_stride < 2 * (int64_t)G2 && sm_frame_abs < n * (int64_t)G2))
    return fail(FFMP_E_ARG, "state_m strides overlap: env %lld, frame %lld elements (G*G = %d)",
                (long long)sm_stride, (long long)sm_frame, G2);
  const int32_t newest = (flags & FFMP_RASTER_NEWEST) ? 1 : 0;
  // 2-D wave tiles: R rows x 256/R columns, where the plane and the block split into them
  const int fmt = raster_format(ct, cfg->grid, flags);
  // 2-D wave tiles: R rows x (cells per wave task)/R columns, where the plane and the block split into them
  int32_t tile_log2r = tile_rows_log2(flags);
  if (tile_log2r) {
    const int C = (fmt == FMT_CT16 ? 1024 : fmt == FMT_CT8 ? 512 : 256) >> tile_log2r, R = 1 << tile_log2r;
    const bool whole_bands = cpb >= G2 || (cpb % (cfg->grid * R)) == 0;
    if ((cfg->grid % C) != 0 || !whole_bands) tile_log2r = 0;  // the 1-D chunks (identical results)
  }
  const dim3 block(256);
  hipStream_t s = (hipStream_t)stream;
  const int64_t rs = rec_stride(cfg->n_obst);
  for (int64_t e0 = 0; e0 < n; e0 += max_envs) {
    const int64_t m = n - e0 < max_envs ? n - e0 : max_envs;
    const dim3 grid((unsigned)(m * bpe));
    const float* rec = record + e0 * rs;
    const uint8_t* msk = mask ? mask + e0 : nullptr;
    float* sm = (float*)((char*)obs->state_m + e0 * sm_stride * (ct ? 1 : 4));
    float* pot = obs->potential ? (float*)((char*)obs->potential + e0 * (int64_t)G2 * (ct ? 2 : 4)) : nullptr;
    float* flw = obs->flow ? (float*)((char*)obs->flow + e0 * 2 * (int64_t)G2 * (ct ? 2 : 4)) : nullptr;
    dispatch_variant(fmt, nt, xcd, fl, [&](auto NT_, auto XCD_, auto FL_, auto FMT_) {
      hipLaunchKernelGGL((raster_kernel<decltype(NT_)::value, decltype(XCD_)::value, decltype(FL_)::value, decltype(FMT_)::value>), grid, block, tuning().lds_pad, s, *cfg, m,
                         bpe, cpb, rec, msk, sm, sm_stride, sm_frame, newest, pot, flw, tile_log2r);
    });
    if (int rc2 = check_launch("ffmp_raster")) return rc2;
  }
  return FFMP_OK;
}

int ffmp_raster(const ffmp_cfg_t* cfg, int64_t n, const float* record, const uint8_t* mask, ffmp_obs_t* obs,
                void* stream) {
  const Tuning& tu = tuning();
  const int32_t flags = (tu.nontemporal == 1 ? FFMP_RASTER_NT : tu.nontemporal == 0 ? FFMP_RASTER_PLAIN : 0) |
                        (tu.xcd_remap ? FFMP_RASTER_XCD : 0);
  return ffmp_raster_ex(cfg, n, record, mask, obs, tu.cells_per_block, flags, stream);
}

int ffmp_step(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset, const int64_t* action,
              ffmp_state_t* state, ffmp_obs_t* obs, ffmp_out_t* out, void* stream) {
  int rc = ffmp_step_state(cfg, n, env_offset, action, state, obs, out, stream);
  if (rc) return rc;
  return ffmp_raster(cfg, n, state->record, nullptr, obs, stream);
}

int ffmp_step_fused(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset, const int64_t* action,
                    ffmp_state_t* state, ffmp_obs_t* obs, ffmp_out_t* out, int32_t flags, void* stream) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (n < 0 || env_offset < 0) return fail(FFMP_E_ARG, "negative n or env_offset");
  if (!state || !obs || !action || !out) return fail(FFMP_E_ARG, "state/obs/action/out is NULL");
  if (!state->pose || !state->goal || !state->d0 || !state->t || !state->episode || !state->record || !state->err)
    return fail(FFMP_E_ARG, "a state pointer is NULL");
  if (cfg->n_obst > 0 && (!state->obst || !state->obst_r)) return fail(FFMP_E_ARG, "obstacle state NULL");
  if (!obs->state_m || !obs->state_g || !obs->state_v || !obs->state_t || !obs->grad)
    return fail(FFMP_E_ARG, "an obs pointer is NULL");
  if (cfg->n_beams > 0 && !obs->lidar) return fail(FFMP_E_ARG, "obs.lidar NULL with n_beams > 0");
  if (!out->reward || !out->done || !out->is_goal || !out->collide || !out->truncated)
    return fail(FFMP_E_ARG, "an out pointer is NULL");
  if ((flags & FFMP_RASTER_NT) && (flags & FFMP_RASTER_PLAIN)) return fail(FFMP_E_ARG, "NT and PLAIN both set");
  const bool fl = cfg->flow != 0;
  if (fl && !obs->flow) return fail(FFMP_E_ARG, "cfg.flow is set but obs.flow is NULL");
  if (int rc2 = check_format(obs, fl)) return rc2;
  const bool ct = obs->format == FFMP_OBS_U8F16;
  if (n == 0) return FFMP_OK;
  if (n > 0x7fffffffLL / 256) return fail(FFMP_E_ARG, "n too large for one launch: %lld", (long long)n);  // one block per env
  const int G2 = cfg->grid * cfg->grid;
  const int64_t sm_stride = obs->state_m_stride ? obs->state_m_stride : 2 * (int64_t)G2;
  const int64_t sm_frame = obs->state_m_frame_stride ? obs->state_m_frame_stride : (int64_t)G2;
  const int64_t sm_frame_abs = sm_frame < 0 ? -sm_frame : sm_frame;  // negative: newest in a lower slot
  if (sm_stride < (int64_t)G2 || sm_frame_abs < (int64_t)G2 ||
      (sm_stride < 2 * (int64_t)G2 && sm_frame_abs < n * (int64_t)G2))
    return fail(FFMP_E_ARG, "state_m strides overlap: env %lld, frame %lld elements (G*G = %d)", (long long)sm_stride,
                (long long)sm_frame, G2);
  const bool nt = (flags & FFMP_RASTER_NT) ? true : (flags & FFMP_RASTER_PLAIN) ? false : (G2 <= 16384);
  const bool xcd = (flags & FFMP_RASTER_XCD) != 0;
  const int32_t newest = (flags & FFMP_RASTER_NEWEST) ? 1 : 0;
  const int fmt = raster_format(ct, cfg->grid, flags);
  int32_t tile_log2r = tile_rows_log2(flags);
  if (tile_log2r && (cfg->grid % ((fmt == FMT_CT16 ? 1024 : fmt == FMT_CT8 ? 512 : 256) >> tile_log2r)) != 0)
    tile_log2r = 0;  // a block is one whole plane
  const dim3 grid((unsigned)n), block(256);
  hipStream_t s = (hipStream_t)stream;
  ffmp_out_t o = *out;
  dispatch_variant(fmt, nt, xcd, fl, [&](auto NT_, auto XCD_, auto FL_, auto FMT_) {
    hipLaunchKernelGGL((step_raster_kernel<decltype(NT_)::value, decltype(XCD_)::value, decltype(FL_)::value, decltype(FMT_)::value>), grid, block, tuning().lds_pad, s, *cfg, n,
                       env_offset, action, *state, *obs, o, sm_stride, sm_frame, newest, tile_log2r);
  });
  return check_launch("ffmp_step_fused");
}

#ifndef FFMP_SKEW_ENV_SPAN
// the share of the raster's blocks the env blocks are spread over: 0 = all dispatched first.  Spread
// over the first quarter / half / 90 % they slowed the raster beside them (C3 13.3-13.5 M against
// 13.9 front-loaded; C2 no better; profiles/r05s_skew_span.txt)
#define FFMP_SKEW_ENV_SPAN 0.0
#endif
static constexpr double kSkewEnvSpan = FFMP_SKEW_ENV_SPAN;

// ffmp_step_skewed; dry_run: every check (the LDS fit included), no launch (ffmp_step_skewed_check)
static int step_skewed(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset, const int64_t* action_next,
                       ffmp_state_t* state_next, ffmp_obs_t* obs, ffmp_out_t* out, const float* record_raster,
                       int32_t cells_per_block, int32_t flags, void* stream, bool dry_run) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (n < 0 || env_offset < 0) return fail(FFMP_E_ARG, "negative n or env_offset");
  if (!state_next || !obs || !action_next || !out || !record_raster)
    return fail(FFMP_E_ARG, "state/obs/action/out/record_raster is NULL");
  if (!state_next->pose || !state_next->goal || !state_next->d0 || !state_next->t || !state_next->episode ||
      !state_next->record || !state_next->err)
    return fail(FFMP_E_ARG, "a state pointer is NULL");
  if (state_next->record == record_raster)
    return fail(FFMP_E_ARG, "ffmp_step_skewed: the env step must write the other record buffer");
  if (cfg->n_obst > 0 && (!state_next->obst || !state_next->obst_r)) return fail(FFMP_E_ARG, "obstacle state NULL");
  if (!obs->state_m || !obs->state_g || !obs->state_v || !obs->state_t || !obs->grad)
    return fail(FFMP_E_ARG, "an obs pointer is NULL");
  if (cfg->n_beams > 0 && !obs->lidar) return fail(FFMP_E_ARG, "obs.lidar NULL with n_beams > 0");
  if (!out->reward || !out->done || !out->is_goal || !out->collide || !out->truncated)
    return fail(FFMP_E_ARG, "an out pointer is NULL");
  if ((flags & FFMP_RASTER_NT) && (flags & FFMP_RASTER_PLAIN)) return fail(FFMP_E_ARG, "NT and PLAIN both set");
  if (cells_per_block != 0 && (cells_per_block < 1024 || cells_per_block % 1024 != 0))
    return fail(FFMP_E_ARG, "cells_per_block must be 0 or a multiple of 1024, got %d", cells_per_block);
  if (int rc2 = check_format(obs, cfg->flow != 0)) return rc2;
  // the instances there are: float32 frames, no flow planes, one disc per lane on 8..64 lanes
  if (obs->format != FFMP_OBS_F32 || cfg->flow) return fail(FFMP_E_ARG, "ffmp_step_skewed: float32 frames without flow planes only");
  const int lpe = cfg->n_obst <= 8 ? 8 : cfg->n_obst <= 16 ? 16 : cfg->n_obst <= 32 ? 32 : 64;
  if (n == 0) return FFMP_OK;
  const int G2 = cfg->grid * cfg->grid;
  const int cpb_max = cells_per_block ? cells_per_block : 4096;
  const int cpb = G2 < cpb_max ? ((G2 + 1023) / 1024) * 1024 : cpb_max;
  const int bpe = (G2 + cpb - 1) / cpb;
  const int64_t env_per_block = 4 * (64 / lpe);
  const int64_t env_chunks = ((n + env_per_block - 1) / env_per_block + 7) / 8;  // 8 env blocks each
  const int64_t ras_blocks = n * bpe;
  // the env blocks spread over the first kSkewEnvSpan of the raster's blocks
  const int64_t chunk_s = std::max<int64_t>(0, (int64_t)(kSkewEnvSpan * (double)ras_blocks) / (8 * env_chunks));
  if (ras_blocks + 8 * env_chunks > 0x7fffffffLL / 256) return fail(FFMP_E_ARG, "ffmp_step_skewed: n too large for one launch");
  if (env_chunks * 8 * chunk_s > ras_blocks) return fail(FFMP_E_ARG, "ffmp_step_skewed: block layout");
  const int64_t sm_stride = obs->state_m_stride ? obs->state_m_stride : 2 * (int64_t)G2;
  const int64_t sm_frame = obs->state_m_frame_stride ? obs->state_m_frame_stride : (int64_t)G2;
  const int64_t sm_frame_abs = sm_frame < 0 ? -sm_frame : sm_frame;
  if (sm_stride < (int64_t)G2 || sm_frame_abs < (int64_t)G2 ||
      (sm_stride < 2 * (int64_t)G2 && sm_frame_abs < n * (int64_t)G2))
    return fail(FFMP_E_ARG, "state_m strides overlap: env %lld, frame %lld elements (G*G = %d)", (long long)sm_stride,
                (long long)sm_frame, G2);
  const bool nt = (flags & FFMP_RASTER_NT) ? true : (flags & FFMP_RASTER_PLAIN) ? false : (G2 <= 16384);
  const bool xcd = (flags & FFMP_RASTER_XCD) != 0;
  const int32_t newest = (flags & FFMP_RASTER_NEWEST) ? 1 : 0;
  int32_t tile_log2r = tile_rows_log2(flags);
  if (tile_log2r) {
    const int C = 256 >> tile_log2r, R = 1 << tile_log2r;
    const bool whole_bands = cpb >= G2 || (cpb % (cfg->grid * R)) == 0;
    if ((cfg->grid % C) != 0 || !whole_bands) tile_log2r = 0;
  }
  const size_t keys = (size_t)4 * (64 / lpe) * (size_t)cfg->n_beams * sizeof(uint32_t);
  const dim3 grid((unsigned)(ras_blocks + 8 * env_chunks)), block(256);
  hipStream_t s = (hipStream_t)stream;
  ffmp_out_t o = *out;
  auto go = [&](auto NT_, auto XCD_, auto L_) {
    constexpr bool kNT = decltype(NT_)::value, kXCD = decltype(XCD_)::value;
    constexpr int kL = decltype(L_)::value;
    static const size_t static_lds = [] {
      hipFuncAttributes a{};
      return hipFuncGetAttributes(&a, reinterpret_cast<const void*>(&skew_kernel<kNT, kXCD, kL>)) == hipSuccess
                 ? (size_t)a.sharedSizeBytes
                 : (size_t)0;
    }();
    if (static_lds + keys > device_lds_limit()) return false;
    if (dry_run) return true;
    hipLaunchKernelGGL((skew_kernel<kNT, kXCD, kL>), grid, block, keys, s, *cfg, n, env_offset, action_next, *state_next,
                       *obs, o, (int32_t)env_chunks, (int32_t)chunk_s, bpe, cpb, record_raster, sm_stride, sm_frame,
                       newest, tile_log2r);
    return true;
  };
  using T = std::true_type;
  using N = std::false_type;
  auto with_l = [&](auto NT_, auto XCD_) {
    switch (lpe) {
      case 8: return go(NT_, XCD_, std::integral_constant<int, 8>{});
      case 16: return go(NT_, XCD_, std::integral_constant<int, 16>{});
      case 32: return go(NT_, XCD_, std::integral_constant<int, 32>{});
      default: return go(NT_, XCD_, std::integral_constant<int, 64>{});
    }
  };
  const bool ok = nt ? (xcd ? with_l(T{}, T{}) : with_l(T{}, N{})) : (xcd ? with_l(N{}, T{}) : with_l(N{}, N{}));
  if (!ok) return fail(FFMP_E_ARG, "ffmp_step_skewed: the env waves' LDS does not fit (L = %d)", cfg->n_beams);
  if (dry_run) return FFMP_OK;
  return check_launch("ffmp_step_skewed");
}

int ffmp_step_skewed(const ffmp_cfg_t* cfg, int64_t n, int64_t env_offset, const int64_t* action_next,
                     ffmp_state_t* state_next, ffmp_obs_t* obs, ffmp_out_t* out, const float* record_raster,
                     int32_t cells_per_block, int32_t flags, void* stream) {
  return step_skewed(cfg, n, env_offset, action_next, state_next, obs, out, record_raster, cells_per_block, flags,
                     stream, false);
}

int ffmp_step_skewed_check(const ffmp_cfg_t* cfg, int32_t format, int32_t flags) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (format != FFMP_OBS_F32 || cfg->flow) return fail(FFMP_E_ARG, "ffmp_step_skewed: float32 frames without flow planes only");
  if (cfg->n_obst > FFMP_MAX_OBST) return fail(FFMP_E_ARG, "n_obst > FFMP_MAX_OBST");
  // the launch's own checks on a placeholder batch of one env, stopped before the launch
  static double dummy[8];
  static float fdummy[64];
  static int32_t idummy[2];
  static uint32_t udummy[1];
  static uint8_t bdummy[4];
  static int64_t adummy[1];
  ffmp_state_t st{dummy, dummy, dummy, dummy, dummy, idummy, idummy, fdummy, udummy, nullptr, nullptr};
  ffmp_obs_t ob{fdummy, fdummy, fdummy, fdummy, nullptr, fdummy, fdummy, nullptr, 0, 0, FFMP_OBS_F32, 0};
  ffmp_out_t o{fdummy, bdummy, bdummy + 1, bdummy + 2, bdummy + 3};
  return step_skewed(cfg, 1, 0, adummy, &st, &ob, &o, fdummy + 32, 0, flags & ~FFMP_RASTER_NEWEST, nullptr, true);
}

int ffmp_reward_done(const ffmp_cfg_t* cfg, int64_t n, const double* scan, int32_t scan_len,
                     const float* local_map, int64_t map_stride, const uint8_t* collide_in,
                     const uint8_t* goal_in, const double* rel_goal, const uint8_t* is_first,
                     double* d0, double* reward, uint8_t* done, uint8_t* is_goal, uint8_t* collide,
                     void* stream) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (n < 0 || scan_len < 0) return fail(FFMP_E_ARG, "negative n or scan_len");
  if (!rel_goal || !is_first || !d0 || !reward || !done || !is_goal || !collide)
    return fail(FFMP_E_ARG, "a required pointer is NULL");
  if (n == 0) return FFMP_OK;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  hipLaunchKernelGGL(reward_done_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, *cfg, n, scan,
                     scan_len, local_map, map_stride, collide_in, goal_in, rel_goal, is_first, d0, reward,
                     done, is_goal, collide);
  return check_launch("ffmp_reward_done");
}

int ffmp_reward_done_packed(const ffmp_cfg_t* cfg, void* host_buf, void* dev_buf, int64_t in_bytes, int32_t scan_len,
                            int64_t map_off, int32_t map_grid, int32_t flags, void* stream) {
  if (!host_buf || !dev_buf) return fail(FFMP_E_ARG, "ffmp_reward_done_packed: NULL buffer");
  if (scan_len < 0 || in_bytes < 48 + 8 * (int64_t)scan_len)
    return fail(FFMP_E_ARG, "ffmp_reward_done_packed: %lld bytes cannot hold %d beams", (long long)in_bytes, scan_len);
  const bool with_map = flags & 4;
  if (with_map && (map_grid <= 0 || map_off < 48 + 8 * (int64_t)scan_len || map_off % 16 ||
                   map_off + 4 * (int64_t)map_grid * map_grid > in_bytes))
    return fail(FFMP_E_ARG, "ffmp_reward_done_packed: map of %d^2 at byte %lld outside the %lld-byte buffer", map_grid,
                (long long)map_off, (long long)in_bytes);
  if (((uintptr_t)host_buf | (uintptr_t)dev_buf) & 15) return fail(FFMP_E_ARG, "ffmp_reward_done_packed: buffers must be 16-byte aligned");
  const hipStream_t s = (hipStream_t)stream;
  if ((flags & 8) && !with_map && scan_len <= FFMP_PACKED_ARG_BEAMS) {
    // inputs as kernel arguments, outputs into the pinned block itself: one launch and a synchronize
    void* out_dev = nullptr;
    if (hipHostGetDevicePointer(&out_dev, host_buf, 0) == hipSuccess && out_dev) {
      if (int rc = check_cfg(cfg)) return rc;
      const char* h = (const char*)host_buf;
      PackedArgs a;
      memcpy(a.scan, h + 48, 8 * (size_t)scan_len);
      memcpy(&a.dist, h + 24, 8);
      memcpy(&a.d0, h + 8, 8);
      a.robot_r = cfg->robot_r;
      a.goal_thr = cfg->goal_thr;
      a.scan_len = scan_len;
      a.is_first = (uint8_t)h[40];
      a.collide_in = (uint8_t)h[41];
      a.goal_in = (uint8_t)h[42];
      a.flags = (uint8_t)(flags & 3);
      hipLaunchKernelGGL(reward_done_args_kernel, dim3(1), dim3(64), 0, s, a, (uint8_t*)out_dev);
      if (int rc = check_launch("ffmp_reward_done_packed")) return rc;
      const hipError_t e = hipStreamSynchronize(s);
      if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_reward_done_packed: %s", hipGetErrorString(e));
      return FFMP_OK;
    }
    (void)hipGetLastError();  // not a mapped host block: the copies below
  }
  if (hipMemcpyAsync(dev_buf, host_buf, (size_t)in_bytes, hipMemcpyHostToDevice, s) != hipSuccess)
    return fail(FFMP_E_HIP, "ffmp_reward_done_packed: host -> device copy failed");
  char* d = (char*)dev_buf;
  uint8_t* u = (uint8_t*)dev_buf;
  const int rc = ffmp_reward_done(cfg, 1, scan_len ? (const double*)(d + 48) : nullptr, scan_len,
                                  with_map ? (const float*)(d + map_off) : nullptr, (int64_t)map_grid * map_grid,
                                  (flags & 1) ? u + 41 : nullptr, (flags & 2) ? u + 42 : nullptr, (const double*)(d + 24),
                                  u + 40, (double*)(d + 8), (double*)d, u + 16, u + 17, u + 18, stream);
  if (rc) return rc;
  if (hipMemcpyAsync(host_buf, dev_buf, 24, hipMemcpyDeviceToHost, s) != hipSuccess)
    return fail(FFMP_E_HIP, "ffmp_reward_done_packed: device -> host copy failed");
  const hipError_t e = hipStreamSynchronize(s);
  if (e != hipSuccess) return fail(FFMP_E_HIP, "ffmp_reward_done_packed: %s", hipGetErrorString(e));
  return FFMP_OK;
}

int ffmp_footprint_collision(const ffmp_cfg_t* cfg, int64_t n, const float* local_map, int64_t map_stride,
                             uint8_t* collide, void* stream) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (n < 0) return fail(FFMP_E_ARG, "negative n");
  if (!local_map || !collide) return fail(FFMP_E_ARG, "local_map/collide is NULL");
  if (n == 0) return FFMP_OK;
  hipLaunchKernelGGL(footprint_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     *cfg, n, local_map, map_stride, collide);
  return check_launch("ffmp_footprint_collision");
}

int ffmp_scan_collision(int64_t n, int32_t L, const float* ranges, double thr, uint8_t* collide, float* min_r,
                        void* stream) {
  return scan_impl<float>(n, L, ranges, thr, collide, min_r, stream);
}

int ffmp_scan_collision_f64(int64_t n, int32_t L, const double* ranges, double thr, uint8_t* collide,
                            double* min_r, void* stream) {
  return scan_impl<double>(n, L, ranges, thr, collide, min_r, stream);
}

int ffmp_check_exact_math(int32_t which, uint32_t lo_bits, uint32_t hi_bits, unsigned long long* mismatches,
                          uint32_t* first_bits, void* stream) {
  if (which != 0 && which != 1) return fail(FFMP_E_ARG, "which must be 0 (sqrt) or 1 (rcp), got %d", which);
  if (!mismatches || !first_bits) return fail(FFMP_E_ARG, "mismatches/first_bits is NULL");
  if (hi_bits <= lo_bits) return FFMP_OK;
  const uint64_t n = (uint64_t)hi_bits - lo_bits;
  const unsigned blocks = (unsigned)std::min<uint64_t>((n + 255) / 256, 65536);
  hipLaunchKernelGGL(exact_math_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, which, lo_bits, hi_bits,
                     mismatches, first_bits);
  return check_launch("ffmp_check_exact_math");
}

int ffmp_episode_init(int64_t n, const uint8_t* mask, int32_t flags, ffmp_episode_t* ep, void* stream) {
  if (n < 0) return fail(FFMP_E_ARG, "negative n");
  if (const int rc = check_episode(ep)) return rc;
  if (ep->totals && !mask &&
      hipMemsetAsync(ep->totals, 0, sizeof(uint64_t) * FFMP_EP_TOTALS, (hipStream_t)stream) != hipSuccess)
    return fail(FFMP_E_HIP, "ffmp_episode_init: hipMemsetAsync failed");
  if (n == 0) return FFMP_OK;
  hipLaunchKernelGGL(episode_init_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, n,
                     mask, flags, *ep);
  return check_launch("ffmp_episode_init");
}

int ffmp_episode_update(int64_t n, const ffmp_out_t* out, int32_t window, int32_t max_steps, double threshold,
                        int32_t flags, ffmp_episode_t* ep, void* stream) {
  if (n < 0) return fail(FFMP_E_ARG, "negative n");
  if (window < 1 || window > 64) return fail(FFMP_E_ARG, "window must be in [1, 64], got %d", window);
  if (max_steps < 0) return fail(FFMP_E_ARG, "negative max_steps");
  if (!out || !out->done || !out->is_goal || !out->collide || !out->truncated)
    return fail(FFMP_E_ARG, "out or one of its flag arrays is NULL");
  if (const int rc = check_episode(ep)) return rc;
  if (n == 0) return FFMP_OK;
  hipLaunchKernelGGL(episode_update_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     n, *out, window, max_steps, threshold, flags, *ep);
  return check_launch("ffmp_episode_update");
}

int ffmp_temporal_maps(int64_t n, const void* frames, const int64_t* lag_offset, int32_t k, int64_t env_stride,
                       int64_t plane, int32_t elem_bytes, const int32_t* since, void* out, void* stream) {
  if (n < 0) return fail(FFMP_E_ARG, "negative n");
  if (k < 1 || k > FFMP_MAX_SERIES) return fail(FFMP_E_ARG, "k must be in [1, %d], got %d", FFMP_MAX_SERIES, k);
  if (elem_bytes != 1 && elem_bytes != 2 && elem_bytes != 4)
    return fail(FFMP_E_ARG, "elem_bytes must be 1, 2 or 4, got %d", elem_bytes);
  if (plane <= 0 || env_stride < 0) return fail(FFMP_E_ARG, "plane must be > 0 and env_stride >= 0");
  if (n == 0) return FFMP_OK;
  if (!frames || !lag_offset || !out) return fail(FFMP_E_ARG, "frames/lag_offset/out is NULL");
  const int64_t plane_b = plane * elem_bytes, env_b = env_stride * elem_bytes;
  if (plane_b % 16 || env_b % 16 || ((uintptr_t)frames % 16) || ((uintptr_t)out % 16))
    return fail(FFMP_E_ARG, "frames, out, the plane (%lld B) and env stride (%lld B) must be 16-byte aligned",
                (long long)plane_b, (long long)env_b);
  LagOffsets lag;
  for (int d = 0; d < FFMP_MAX_SERIES; ++d) {
    lag.b[d] = lag_offset[std::min(d, k - 1)] * elem_bytes;
    if (lag.b[d] % 16) return fail(FFMP_E_ARG, "lag offset %d is not 16-byte aligned", d);
  }
  const int64_t chunks = (plane_b / 16 + 1023) / 1024;
  if (n * k * chunks > 0x7fffffffLL) return fail(FFMP_E_ARG, "too many blocks for one launch");
  hipLaunchKernelGGL(temporal_maps_kernel, dim3((unsigned)(n * k * chunks)), dim3(256), 0, (hipStream_t)stream,
                     (const char*)frames, lag, k, env_b, plane_b, since, (int32_t)chunks, (char*)out);
  return check_launch("ffmp_temporal_maps");
}

int ffmp_bev_image(int64_t n, int32_t compact, const void* occ, int64_t occ_env_stride, const void* flow,
                   int64_t plane, float vmax, void* out, int64_t out_env_stride, void* stream) {
  if (n < 0) return fail(FFMP_E_ARG, "negative n");
  if (plane <= 0 || occ_env_stride < plane || out_env_stride < 4 * plane)
    return fail(FFMP_E_ARG, "plane must be > 0, occ_env_stride >= plane and out_env_stride >= 4 * plane");
  if (!(vmax > 0.0f) || !std::isfinite(vmax)) return fail(FFMP_E_ARG, "vmax must be finite and > 0");
  if (compact != 0 && compact != 1) return fail(FFMP_E_ARG, "compact must be 0 or 1");
  if (n == 0) return FFMP_OK;
  if (!occ || !flow || !out) return fail(FFMP_E_ARG, "occ/flow/out is NULL");
  const bool quad = plane % 4 == 0 && occ_env_stride % 4 == 0 && out_env_stride % 4 == 0;
  const int64_t per = quad ? 1024 : 256;  // cells per block
  const int64_t chunks = (plane + per - 1) / per;
  if (n * chunks > 0x7fffffffLL) return fail(FFMP_E_ARG, "too many blocks for one launch");
  const dim3 grid((unsigned)(n * chunks));
  hipStream_t s = (hipStream_t)stream;
  if (compact && quad)
    hipLaunchKernelGGL((bev_image_kernel<true, 4>), grid, dim3(256), 0, s, n, occ, occ_env_stride, flow, plane,
                       (int32_t)chunks, vmax, out, out_env_stride);
  else if (compact)
    hipLaunchKernelGGL((bev_image_kernel<true, 1>), grid, dim3(256), 0, s, n, occ, occ_env_stride, flow, plane,
                       (int32_t)chunks, vmax, out, out_env_stride);
  else if (quad)
    hipLaunchKernelGGL((bev_image_kernel<false, 4>), grid, dim3(256), 0, s, n, occ, occ_env_stride, flow, plane,
                       (int32_t)chunks, vmax, out, out_env_stride);
  else
    hipLaunchKernelGGL((bev_image_kernel<false, 1>), grid, dim3(256), 0, s, n, occ, occ_env_stride, flow, plane,
                       (int32_t)chunks, vmax, out, out_env_stride);
  return check_launch("ffmp_bev_image");
}

int ffmp_policy_reactive(const ffmp_cfg_t* cfg, int64_t n, const ffmp_obs_t* obs, int64_t* action, void* stream) {
  int rc = check_cfg(cfg);
  if (rc) return rc;
  if (n < 0) return fail(FFMP_E_ARG, "negative n");
  if (!obs || !obs->state_m || !obs->state_g || !action) return fail(FFMP_E_ARG, "obs.state_m / obs.state_g / action is NULL");
  if (obs->format != FFMP_OBS_F32 && obs->format != FFMP_OBS_U8F16) return fail(FFMP_E_ARG, "unknown obs format %d", obs->format);
  if (n == 0) return FFMP_OK;
  const int64_t G2 = (int64_t)cfg->grid * cfg->grid;
  const int64_t env_stride = obs->state_m_stride ? obs->state_m_stride : 2 * G2;
  const int64_t frame = obs->state_m_frame_stride ? obs->state_m_frame_stride : G2;
  // the look-ahead ray: from just outside the footprint (3 cells) to ~0.4 m ahead, inside the map
  const int32_t look0 = 3, look1 = std::min<int32_t>(3 + (int32_t)std::lround(0.25 / cfg->res), cfg->grid / 2 - 1);
  if (look1 < look0) return fail(FFMP_E_ARG, "grid %d too small for the look-ahead", cfg->grid);
  const dim3 grid((unsigned)((n + 255) / 256)), block(256);
  hipStream_t s = (hipStream_t)stream;
  if (obs->format == FFMP_OBS_F32)
    hipLaunchKernelGGL(policy_reactive_kernel<float>, grid, block, 0, s, n, cfg->grid, obs->state_m + frame, env_stride,
                       obs->state_g, look0, look1, 1.0f, action);
  else
    hipLaunchKernelGGL(policy_reactive_kernel<uint8_t>, grid, block, 0, s, n, cfg->grid,
                       reinterpret_cast<const uint8_t*>(obs->state_m) + frame, env_stride, obs->state_g, look0, look1,
                       1.0f, action);
  return check_launch("ffmp_policy_reactive");
}

#ifdef FFMP_TRACE
// Probe builds only: copy the stamps (env: 4096 x 12, raster: 65536 x 4 uint64) to host memory.
int ffmp_trace_read(uint64_t* env_host, uint64_t* ras_host, int clear) {
  if (hipMemcpyFromSymbol(env_host, HIP_SYMBOL(g_trace_env), sizeof(uint64_t) * 4096 * 12) != hipSuccess ||
      hipMemcpyFromSymbol(ras_host, HIP_SYMBOL(g_trace_ras), sizeof(uint64_t) * 65536 * 4) != hipSuccess)
    return fail(FFMP_E_HIP, "ffmp_trace_read: copy failed");
  if (clear) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_trace_env)) != hipSuccess || hipMemset(p, 0, sizeof(uint64_t) * 4096 * 12) != hipSuccess ||
        hipGetSymbolAddress(&p, HIP_SYMBOL(g_trace_ras)) != hipSuccess || hipMemset(p, 0, sizeof(uint64_t) * 65536 * 4) != hipSuccess)
      return fail(FFMP_E_HIP, "ffmp_trace_read: clear failed");
  }
  return hipDeviceSynchronize() == hipSuccess ? FFMP_OK : fail(FFMP_E_HIP, "ffmp_trace_read: sync failed");
}
#endif
}  // extern "C"
