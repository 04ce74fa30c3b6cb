// ffmp_device.h — device-side building blocks of the batched FFMP step.
//
// Arithmetic contract (mirrored operation-for-operation by oracle/ffmp_oracle.py;
// compile with -ffp-contract=off so no a*b+c is fused):
//   * per-env scalars (pose, goal, obstacles, lidar, reward) in float64, like
//     the reference's Python floats (src/train.py:167-188, ffmp.py:130-157);
//   * per-cell raster maths in float32 (the BEV planes are float32 tensors,
//     src/train.py:116-121, :543-545).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include "../../include/ffmp.h"

#pragma clang fp contract(off)

#define FFMP_DEV __device__ __forceinline__

namespace ffmp {

constexpr double kPi = 3.141592653589793;       // math.pi
constexpr double kTwoPi = 2.0 * 3.141592653589793;  // 2 * math.pi (train.py:169)
constexpr double kInv2p32 = 2.3283064365386962890625e-10;  // 2^-32

// RobotAction.cmd (src/gym_ffmp/envs/robot/config.py:28-55): id = 7*vi + wi.
// The literal lists, never computed (0.6 != 3*0.2 in binary) — as selects over immediate
// operands rather than a __constant__ table: a per-lane table index is a vector load, one more
// dependent memory round trip at the head of the env step's latency chain.
FFMP_DEV double cmd_v(int vi) { return vi == 0 ? 0.0 : vi == 1 ? 0.2 : vi == 2 ? 0.4 : 0.6; }
FFMP_DEV double cmd_w(int wi) {
  return wi == 0 ? -0.6 : wi == 1 ? -0.4 : wi == 2 ? -0.2 : wi == 3 ? 0.0 : wi == 4 ? 0.2 : wi == 5 ? 0.4 : 0.6;
}

// ROSNode.pi_to_pi (src/train.py:167-172): iterative wrap into (-pi, pi].
// (+-inf would loop forever in the reference; returned unchanged here.)
FFMP_DEV double pi_to_pi(double a) {
  if (!(a - a == 0.0)) return a;  // inf / nan
  while (a >= kPi) a = a - kTwoPi;
  while (a <= -kPi) a = a + kTwoPi;
  return a;
}

// ---------------- Philox4x32-10 (Salmon et al., SC'11) ----------------------
struct U4 { uint32_t x, y, z, w; };

FFMP_DEV U4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                          uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
    const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
    const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
    c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
    k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
  }
  return U4{c0, c1, c2, c3};
}

// counter = (draw index, episode, global env lo, global env hi), key = seed.
FFMP_DEV U4 draw(const ffmp_cfg_t& cfg, int64_t genv, int32_t episode, uint32_t idx) {
  const uint64_t g = (uint64_t)genv;
  return philox4x32_10(idx, (uint32_t)episode, (uint32_t)g, (uint32_t)(g >> 32),
                       (uint32_t)cfg.seed, (uint32_t)(cfg.seed >> 32));
}
FFMP_DEV double u01(uint32_t r) { return (double)r * kInv2p32; }

// Draw-index layout of one episode's reset.
constexpr uint32_t kDrawObst = 1;                       // + k*16 + try
constexpr int kObstTries = 16;
constexpr uint32_t kDrawVel = 1 + FFMP_MAX_OBST * kObstTries;  // + k

// ---------------- per-env episode sampling ----------------------------------
struct Episode {
  double x, y, yaw, gx, gy;
};

FFMP_DEV Episode sample_episode(const ffmp_cfg_t& cfg, int64_t genv, int32_t episode) {
  const U4 b = draw(cfg, genv, episode, 0);
  Episode ep;
  ep.x = 0.0;
  ep.y = 0.0;
  ep.yaw = u01(b.x) * kTwoPi - kPi;
  const double gd = cfg.goal_min + u01(b.y) * (cfg.goal_max - cfg.goal_min);
  const double gb = u01(b.z) * kTwoPi - kPi;
  ep.gx = gd * cos(gb);
  ep.gy = gd * sin(gb);
  return ep;
}

struct Obst {
  double x, y, vx, vy, r;
};

FFMP_DEV Obst sample_obstacle(const ffmp_cfg_t& cfg, int64_t genv, int32_t episode, int k,
                              const Episode& ep) {
  const double W = cfg.world_half;
  Obst o;
  bool ok = false;
  for (int tr = 0; tr < kObstTries && !ok; ++tr) {
    const U4 b = draw(cfg, genv, episode, kDrawObst + (uint32_t)(k * kObstTries + tr));
    o.r = cfg.obst_rmin + u01(b.z) * (cfg.obst_rmax - cfg.obst_rmin);
    const double span = 2.0 * (W - o.r);
    o.x = (o.r - W) + u01(b.x) * span;
    o.y = (o.r - W) + u01(b.y) * span;
    const double ds = o.r + cfg.start_clear, dg = o.r + cfg.goal_clear;
    const double sx = o.x - ep.x, sy = o.y - ep.y;
    const double gx = o.x - ep.gx, gy = o.y - ep.gy;
    ok = (sx * sx + sy * sy > ds * ds) && (gx * gx + gy * gy > dg * dg);
  }
  o.vx = 0.0;
  o.vy = 0.0;
  if (!ok) {  // parked: zero radius far outside the world
    o.x = 3.0 * W;
    o.y = 3.0 * W;
    o.r = 0.0;
  } else if (cfg.moving) {
    const U4 b = draw(cfg, genv, episode, kDrawVel + (uint32_t)k);
    const double sp = u01(b.x) * cfg.obst_vmax;
    const double hd = u01(b.y) * kTwoPi - kPi;
    o.vx = sp * cos(hd);
    o.vy = sp * sin(hd);
  }
  return o;
}

// Obstacle motion with specular reflection off the world walls; parked discs
// (r == 0) stay where they are.
FFMP_DEV void move_obstacle(const ffmp_cfg_t& cfg, Obst& o) {
  if (!(o.r > 0.0)) return;
  const double W = cfg.world_half;
  o.x = o.x + o.vx * cfg.dt;
  if (o.x > W - o.r) { o.x = 2.0 * (W - o.r) - o.x; o.vx = -o.vx; }
  else if (o.x < o.r - W) { o.x = 2.0 * (o.r - W) - o.x; o.vx = -o.vx; }
  o.y = o.y + o.vy * cfg.dt;
  if (o.y > W - o.r) { o.y = 2.0 * (W - o.r) - o.y; o.vy = -o.vy; }
  else if (o.y < o.r - W) { o.y = 2.0 * (o.r - W) - o.y; o.vy = -o.vy; }
}

// ---------------- raster record (per env, float32) ---------------------------
// hdr[0..3] current frame {px, py, cos yaw, sin yaw}; hdr[4..7] previous frame;
// hdr[8..9] goal in the current ego frame; then K float4 {ox, oy, r*r, r} of the
// current frame in ego coordinates, K float4 of the previous frame, and K float4
// {vx, vy, 0, 0}: each disc's velocity rotated into the current ego frame.
struct FrameHdr {
  float px, py, c, s;
};

FFMP_DEV FrameHdr make_hdr(double x, double y, double c, double s) {
  return FrameHdr{(float)x, (float)y, (float)c, (float)s};
}

// World point -> ego frame (float64), rounded to float32.
FFMP_DEV float2 to_ego(double wx, double wy, double x, double y, double c, double s) {
  const double rx = wx - x, ry = wy - y;
  const double ex = c * rx + s * ry;
  const double ey = c * ry - s * rx;
  return make_float2((float)ex, (float)ey);
}

// World velocity -> current ego frame (float64 rotation, rounded to float32).
FFMP_DEV float4 ego_vel(const Obst& o, double c, double s) {
  const double vx = c * o.vx + s * o.vy;
  const double vy = c * o.vy - s * o.vx;
  return make_float4((float)vx, (float)vy, 0.0f, 0.0f);
}

FFMP_DEV float4 ego_obst(const Obst& o, double x, double y, double c, double s) {
  const float2 e = to_ego(o.x, o.y, x, y, c, s);
  const float rf = (float)o.r;
  return make_float4(e.x, e.y, rf * rf, rf);
}

// Ego coordinate of cell index i (row -> ego x, col -> ego y): reference's
// `i * map_grid_size - 0.5 * map_range` (ffmp.py:89-90) in float32.
FFMP_DEV float cell_coord(const ffmp_cfg_t& cfg, int i) {
  return (float)i * cfg.res_f - cfg.half_f;
}

// Outside-the-world test of an ego point (float32).
FFMP_DEV bool outside_world(const ffmp_cfg_t& cfg, const FrameHdr& h, float ex, float ey) {
  const float wx = h.px + (h.c * ex - h.s * ey);
  const float wy = h.py + (h.s * ex + h.c * ey);
  const float W = cfg.world_half_f;
  return (wx < -W) | (wx > W) | (wy < -W) | (wy > W);
}

FFMP_DEV bool in_disc(float ex, float ey, const float4& o) {
  const float dx = ex - o.x, dy = ey - o.y;
  return dx * dx + dy * dy <= o.z;
}

// Repulsive term of one obstacle at an ego point; returns 0 contribution flag.
FFMP_DEV float add_repulsive(const ffmp_cfg_t& cfg, float U, float ex, float ey, const float4& o) {
  const float dx = ex - o.x, dy = ey - o.y;
  float d = sqrtf(dx * dx + dy * dy) - o.w;
  d = fmaxf(d, cfg.rho_min_f);
  if (d < cfg.rho0_f) {
    const float q = 1.0f / d - cfg.inv_rho0_f;
    U = U + cfg.half_kr_f * (q * q);
  }
  return U;
}

// add_repulsive for a cell whose squared distance s = dx*dx + dy*dy to the disc centre is already
// computed (the same float32 operations, so the result is bit-identical), skipping the sqrt and
// the division when s >= reach2 = rep_reach2(cfg, r): there sqrtf(s) - r >= rho0 for certain, so
// the term is exactly zero.
FFMP_DEV float rep_reach2(const ffmp_cfg_t& cfg, float r) {
  const float a = cfg.rho0_f + r;
  return (a * a) * 1.000004f;  // > ((rho0 + r)(1 + 2^-20))^2 despite the rounding of a, a*a and the product
}

// Correctly rounded float32 sqrt for 2^-96 <= s < inf: v_sqrt_f32 (faithful) then the
// neighbour-residual correction — sqrtf without its tiny-input scaling and special-value
// select (16 -> 8 VALU).  Below 2^-96 it may differ from sqrtf, but add_repulsive_s only feeds
// it into fmaxf(sqrt(s) - r, rho_min) with r >= 0 and rho_min >= 2^-48, where both give rho_min.
FFMP_DEV float sqrt_rn(float s) {
  const float y = __builtin_amdgcn_sqrtf(s);
  const float yd = __int_as_float(__float_as_int(y) - 1), yu = __int_as_float(__float_as_int(y) + 1);
  const float rd = __builtin_fmaf(-yd, y, s), ru = __builtin_fmaf(-yu, y, s);
  const float t = (rd <= 0.0f) ? yd : y;
  return (ru > 0.0f) ? yu : t;
}

// Correctly rounded float32 1/d for normal d with 1/d normal: v_rcp_f32 (1 ulp) and one FMA
// Newton step (11 -> 3 VALU).  Both helpers are checked bit-for-bit against sqrtf / 1.0f/d
// over every float of their ranges by ffmp_check_exact_math (tests/test_gpu_exact_math.py).
FFMP_DEV float rcp_rn(float d) {
  const float y = __builtin_amdgcn_rcpf(d);
  const float e = __builtin_fmaf(-d, y, 1.0f);
  return __builtin_fmaf(e, y, y);
}

FFMP_DEV float add_repulsive_s(const ffmp_cfg_t& cfg, float U, float s, float r, float reach2) {
  if (s >= reach2) return U;
  float d = sqrt_rn(s) - r;
  d = fmaxf(d, cfg.rho_min_f);
  if (d < cfg.rho0_f) {
    const float q = rcp_rn(d) - cfg.inv_rho0_f;
    U = U + cfg.half_kr_f * (q * q);
  }
  return U;
}

FFMP_DEV float attractive(const ffmp_cfg_t& cfg, float ex, float ey, float gx, float gy) {
  const float dx = ex - gx, dy = ey - gy;
  return cfg.half_ka_f * (dx * dx + dy * dy);
}

// Potential at cell (i, j) over all K discs — used for the gradient lookup.  The raster's
// arithmetic (add_repulsive_s: the same float32 operations as add_repulsive, skipping discs out
// of repulsive reach), so the gradient is the central difference of the raster's plane.
FFMP_DEV float potential_cell(const ffmp_cfg_t& cfg, const float4* obs, int K, float gx, float gy,
                              int i, int j) {
  const float ex = cell_coord(cfg, i), ey = cell_coord(cfg, j);
  float U = attractive(cfg, ex, ey, gx, gy);
  for (int k = 0; k < K; ++k) {
    const float4 o = obs[k];
    const float dx = ex - o.x, dy = ey - o.y;
    U = add_repulsive_s(cfg, U, dx * dx + dy * dy, o.w, rep_reach2(cfg, o.w));
  }
  return U;
}

FFMP_DEV bool occupied_cell(const ffmp_cfg_t& cfg, const FrameHdr& h, const float4* obs, int K,
                            int i, int j) {
  const float ex = cell_coord(cfg, i), ey = cell_coord(cfg, j);
  bool o = outside_world(cfg, h, ex, ey);
  for (int k = 0; k < K; ++k) o |= in_disc(ex, ey, obs[k]);
  return o;
}

// ---- lidar ------------------------------------------------------------------
// Per-env lidar scene, built lane-parallel once per env (lane k = disc k): the discs that
// can return a hit within lidar_max or contain the sensor, whether the sensor is inside a
// disc, and which walls are within range.  A disc whose surface is farther than
// lidar_max + kLidarCullMargin can never produce an accepted hit (any ray's entry distance is
// >= |rel| - r, and float64 rounding moves the computed value by < 3e-7 m), and likewise a
// wall farther than that (|dir| <= 1), so skipping them leaves every range bit-identical.
constexpr double kLidarCullMargin = 1e-6;

// Ballot over the `lpe` lanes that serve this lane's env (an env owns lanes [g*lpe, g*lpe+lpe) of
// the wave; bit k of the result = its lane k).  lpe is 16, 32 or 64 (wave-uniform).
FFMP_DEV uint64_t group_ballot(bool pred, int lpe) {
  const uint64_t m = __ballot(pred);
  if (lpe == 64) return m;
  const int base = (int)(threadIdx.x & 63) & ~(lpe - 1);
  return (m >> base) & ((1ull << lpe) - 1ull);
}

struct LidarScene {
  uint64_t mask;
  bool inside;
  bool wxp, wxn, wyp, wyn;
};

// Call from every lane of the env's lane group; its lane holds discs k = lane + j lpe (j < DPL),
// those with k < K real.
template <int DPL>
FFMP_DEV LidarScene lidar_scene(const ffmp_cfg_t& cfg, double x, double y, const Obst (&my)[DPL], int lane, int K,
                                int lpe) {
  const double reach = cfg.lidar_max + kLidarCullMargin;
  LidarScene sc;
  sc.mask = 0;
  sc.inside = false;
#pragma unroll
  for (int j = 0; j < DPL; ++j) {
    const bool has = lane + j * lpe < K;
    const double rx = my[j].x - x, ry = my[j].y - y;
    const double rr = rx * rx + ry * ry;
    const bool in = has && (rr <= my[j].r * my[j].r);
    const bool act = has && (in || !(sqrt(rr) - my[j].r > reach));
    sc.mask |= group_ballot(act, lpe) << (j * lpe);
    sc.inside = sc.inside || group_ballot(in, lpe) != 0;
  }
  const double W = cfg.world_half;
  sc.wxp = (W - x) <= reach;
  sc.wxn = (x + W) <= reach;
  sc.wyp = (W - y) <= reach;
  sc.wyn = (y + W) <= reach;
  return sc;
}

// Per-disc lidar operands, written by disc k's lane before the beams (LDS): the disc centre
// relative to the sensor (rx, ry), |rel|^2 and r^2 — the same float64 operations lidar_beam
// did per beam, done once per disc.
FFMP_DEV void lidar_disc(double x, double y, double ox, double oy, double r, double* rxa, double* rya, double* rra,
                         double* r2a, int k) {
  const double rx = ox - x, ry = oy - y;
  rxa[k] = rx;
  rya[k] = ry;
  rra[k] = rx * rx + ry * ry;
  r2a[k] = r * r;
}

// False only if the wall hit h = num / den (num, den of one sign) is certainly beyond L, so the
// float64 division can be skipped without changing any range: |num| > (L*|den|)(1 + 2^-40) in
// float64 means the exact quotient exceeds L(1 + 2^-41), and its rounding stays above L.
FFMP_DEV bool wall_in_reach(double num, double den, double L) {
  return !(fabs(num) > (L * fabs(den)) * (1.0 + 0x1p-40));
}

// One lidar beam (float64): nearest of the scene's discs and walls.  Returns +inf for no
// return within lidar_max, -inf if the origin is inside a disc.  rxa / rya / rra / r2a: the
// scene's discs as lidar_disc wrote them.
FFMP_DEV double lidar_beam(const ffmp_cfg_t& cfg, const LidarScene& sc, double x, double y, double c, double s,
                           double bc, double bs, const double* rxa, const double* rya, const double* rra,
                           const double* r2a) {
  const double inf = __builtin_inf();
  if (sc.inside) return -inf;
  const double dirx = c * bc - s * bs;
  const double diry = s * bc + c * bs;
  double best = inf;
  for (uint64_t m = sc.mask; m; m &= m - 1) {
    const int k = __builtin_ctzll(m);
    const double rx = rxa[k], ry = rya[k];
    const double rr = rra[k];
    const double r2 = r2a[k];
    const double tp = rx * dirx + ry * diry;
    if (tp > 0.0) {
      const double perp = rr - tp * tp;
      if (perp <= r2) {
        const double h = tp - sqrt(r2 - perp);
        if (h <= cfg.lidar_max && h < best) best = h;
      }
    }
  }
  const double W = cfg.world_half, L = cfg.lidar_max;
  if (dirx > 0.0) { if (sc.wxp && wall_in_reach(W - x, dirx, L)) { const double h = (W - x) / dirx; if (h <= L && h < best) best = h; } }
  else if (dirx < 0.0) { if (sc.wxn && wall_in_reach(-W - x, dirx, L)) { const double h = (-W - x) / dirx; if (h <= L && h < best) best = h; } }
  if (diry > 0.0) { if (sc.wyp && wall_in_reach(W - y, diry, L)) { const double h = (W - y) / diry; if (h <= L && h < best) best = h; } }
  else if (diry < 0.0) { if (sc.wyn && wall_in_reach(-W - y, diry, L)) { const double h = (-W - y) / diry; if (h <= L && h < best) best = h; } }
  return best;
}

// CH beams of one lane at a time (beams l0, l0 + lpe, ..., l0 + (CH-1) lpe): the disc loop is
// outermost, so each disc's four LDS operands are read once per CH beams and the CH beams' tests
// are independent chains.  Every beam sees exactly lidar_beam's operations in lidar_beam's order
// (discs in ascending k, then the walls), so every range is bit-identical to it.  The one-launch
// step's env phase uses it; the env kernel traces by discs (trace_discs, below).  (Round 4 tried
// deferring each beam's square root until a second candidate or the loop's end: bit-identical,
// 1-3 us slower at C3, not kept; profiles/r04_env_kernel.txt.)
// f(l, range) for every beam l < n_beams of this lane.
template <int CH, class F>
FFMP_DEV void trace_beams(const ffmp_cfg_t& cfg, const LidarScene& sc, int lane, int lpe, double x, double y,
                          double c, double s, const double* rxa, const double* rya, const double* rra,
                          const double* r2a, F&& f) {
  const double inf = __builtin_inf();
  const double2* bt = reinterpret_cast<const double2*>(cfg.beam_cs);
  const int nb = cfg.n_beams;
  const double W = cfg.world_half, L = cfg.lidar_max;
  for (int l0 = lane; l0 < nb; l0 += CH * lpe) {
    double dirx[CH], diry[CH], best[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int l = l0 + j * lpe;
      const double2 b = l < nb ? bt[l] : make_double2(1.0, 0.0);
      dirx[j] = c * b.x - s * b.y;
      diry[j] = s * b.x + c * b.y;
      best[j] = inf;
    }
    if (!sc.inside) {
      for (uint64_t m = sc.mask; m; m &= m - 1) {
        const int k = __builtin_ctzll(m);
        const double rx = rxa[k], ry = rya[k];
        const double rr = rra[k];
        const double r2 = r2a[k];
#pragma unroll
        for (int j = 0; j < CH; ++j) {
          const double tp = rx * dirx[j] + ry * diry[j];
          if (tp > 0.0) {
            const double perp = rr - tp * tp;
            if (perp <= r2) {
              const double h = tp - sqrt(r2 - perp);
              if (h <= L && h < best[j]) best[j] = h;
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const double dx = dirx[j], dy = diry[j];
        double bj = best[j];
        if (dx > 0.0) { if (sc.wxp && wall_in_reach(W - x, dx, L)) { const double h = (W - x) / dx; if (h <= L && h < bj) bj = h; } }
        else if (dx < 0.0) { if (sc.wxn && wall_in_reach(-W - x, dx, L)) { const double h = (-W - x) / dx; if (h <= L && h < bj) bj = h; } }
        if (dy > 0.0) { if (sc.wyp && wall_in_reach(W - y, dy, L)) { const double h = (W - y) / dy; if (h <= L && h < bj) bj = h; } }
        else if (dy < 0.0) { if (sc.wyn && wall_in_reach(-W - y, dy, L)) { const double h = (-W - y) / dy; if (h <= L && h < bj) bj = h; } }
        best[j] = bj;
      }
    }
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int l = l0 + j * lpe;
      if (l < nb) f(l, sc.inside ? -inf : best[j]);
    }
  }
}

// Order-preserving uint32 key of a float (a < b <=> fkey(a) < fkey(b), NaN aside) for LDS atomic min.
FFMP_DEV uint32_t fkey(float v) {
  const uint32_t b = __float_as_uint(v);
  return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
FFMP_DEV float funkey(uint32_t k) { return __uint_as_float((k & 0x80000000u) ? (k & 0x7fffffffu) : ~k); }

// Disc-major lidar (round 4): the same ranges as lidar_beam / trace_beams, from far fewer tests.
// A disc can return a hit only on the beams within its angular half-width asin(r / |rel|) of its
// centre's bearing; each of the group's discs (lane k = disc k of the scene mask) lists those
// beams — bearing and half-width in float32, widened by 1e-3 rad and one beam on each side —, the
// group's lanes share the (disc, beam) pairs evenly, and each pair runs lidar_beam's exact float64
// test (tp > 0, perp = |rel|^2 - tp^2 <= r^2, h = tp - sqrt(r^2 - perp), h <= lidar_max), its hit
// rounded to float32 joining the beam's minimum by an LDS atomic min.  Then each beam adds its wall
// hits (lidar_beam's tests) and emits.  Identical ranges:
//  * every pair lidar_beam would accept is tested: off the list, a beam's angle to the centre exceeds
//    asin(r/|rel|) by >= 1e-3 rad (the float32 bearing / width / index errors are ~1e-6 rad), so
//    exactly perp - r^2 >= |rel|^2 (sin^2(a + 1e-3) - sin^2 a) >= |rel|^2 1e-6, or tp < 0 by >=
//    |rel| sin(1e-3) past 90 degrees — margins ~10^8 times the float64 rounding of tp and perp;
//    a disc with r^2 / |rel|^2 >= 0.98 lists every beam;
//  * float32 rounding is monotone, so the minimum of the rounded hits (discs and walls) is the
//    rounded minimum lidar_beam returns, and `h <= lidar_max` is decided in float64 per hit as there;
//    h is never -0 (x - x = +0), so the minimum is the same value whatever order the hits arrive in.
// Relies on the beam layout of ffmp_cfg_t.beam_cs (angle -pi + l 2pi/L).  lane / lpe: the env's
// group, holding discs k = lane + j lpe (j < DPL); s_key: the env's L uint32 (LDS), s_pref / s_lo: its
// lpe DPL ints each (LDS).  Every lane of the group calls it (shuffles).  f(l, range) for every beam l.
template <int DPL, class F>
FFMP_DEV void trace_discs(const ffmp_cfg_t& cfg, const LidarScene& sc, int lane, int lpe, double x, double y,
                          double c, double s, const double* rxa, const double* rya, const double* rra,
                          const double* r2a, uint32_t* s_key, int* s_pref, int* s_lo, F&& f) {
  const int nb = cfg.n_beams;
  if (nb <= 0) return;
  const double2* bt = reinterpret_cast<const double2*>(cfg.beam_cs);
  if (sc.inside) {
    for (int l = lane; l < nb; l += lpe) f(l, -__builtin_inf());
    return;
  }
  const double W = cfg.world_half, L = cfg.lidar_max;
  for (int l = lane; l < nb; l += lpe) s_key[l] = fkey(__builtin_inff());
  // this lane's discs k = lane + j lpe: their beams [lo, lo + cnt) (mod L), and the inclusive
  // prefix of the counts over the disc index k (pair p belongs to the first k with s_pref[k] > p)
  int total = 0;
#pragma unroll
  for (int j = 0; j < DPL; ++j) {
    const int k = lane + j * lpe;
    int lo = 0, cnt = 0;
    if ((sc.mask >> k) & 1ull) {
      const double rx = rxa[k], ry = rya[k];
      const float q = (float)(r2a[k] / rra[k]);  // sin^2 of the half-width
      if (!(q < 0.98f)) {
        cnt = nb;
      } else {
        const float ex = (float)(c * rx + s * ry), ey = (float)(c * ry - s * rx);  // the centre, robot frame
        const float th = atan2f(ey, ex);
        const float half = asinf(sqrtf(q)) + 1e-3f;
        const float per = (float)nb * 0.159154943f;  // beams per radian
        lo = (int)floorf((th - half + 3.14159265f) * per) - 1;
        const int hi = (int)ceilf((th + half + 3.14159265f) * per) + 1;
        cnt = min(hi - lo + 1, nb);
        lo %= nb;
        if (lo < 0) lo += nb;
      }
    }
    int incl = cnt;  // inclusive prefix over the group
    for (int o = 1; o < lpe; o <<= 1) {
      const int v = __shfl_up(incl, o, lpe);
      if (lane >= o) incl += v;
    }
    s_pref[k] = total + incl;
    s_lo[k] = lo;
    total += __shfl(incl, lpe - 1, lpe);
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  for (int p = lane; p < total; p += lpe) {
    int k = 0;  // the disc of pair p: the first disc whose inclusive count exceeds p
    for (int step = (lpe * DPL) >> 1; step > 0; step >>= 1)
      if (s_pref[k + step - 1] <= p) k += step;
    int l = s_lo[k] + (p - (k ? s_pref[k - 1] : 0));
    if (l >= nb) l -= nb;
    const double2 b = bt[l];
    const double dirx = c * b.x - s * b.y;
    const double diry = s * b.x + c * b.y;
    const double tp = rxa[k] * dirx + rya[k] * diry;
    if (tp > 0.0) {
      const double perp = rra[k] - tp * tp;
      const double r2 = r2a[k];
      if (perp <= r2) {
        const double h = tp - sqrt(r2 - perp);
        if (h <= L) atomicMin(&s_key[l], fkey((float)h));
      }
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const bool walls = sc.wxp || sc.wxn || sc.wyp || sc.wyn;
  for (int l = lane; l < nb; l += lpe) {
    float r = funkey(s_key[l]);
    if (walls) {
      const double2 b = bt[l];
      const double dx = c * b.x - s * b.y, dy = s * b.x + c * b.y;
      double bj = __builtin_inf();
      if (dx > 0.0) { if (sc.wxp && wall_in_reach(W - x, dx, L)) { const double h = (W - x) / dx; if (h <= L && h < bj) bj = h; } }
      else if (dx < 0.0) { if (sc.wxn && wall_in_reach(-W - x, dx, L)) { const double h = (-W - x) / dx; if (h <= L && h < bj) bj = h; } }
      if (dy > 0.0) { if (sc.wyp && wall_in_reach(W - y, dy, L)) { const double h = (W - y) / dy; if (h <= L && h < bj) bj = h; } }
      else if (dy < 0.0) { if (sc.wyn && wall_in_reach(-W - y, dy, L)) { const double h = (-W - y) / dy; if (h <= L && h < bj) bj = h; } }
      r = fminf(r, (float)bj);
    }
    f(l, (double)r);
  }
}

// FFMP.is_collision2 on one float32 beam (ffmp.py:110-115): `if r:` skips 0,
// `r < ROBOT_RSIZE` is a float64 compare.
FFMP_DEV bool beam_collides(float r, double thr) { return (r != 0.0f) && ((double)r < thr); }

// FFMP.reward_calculator (ffmp.py:130-157), float64, (r_g + r_c) + r_s.
FFMP_DEV double reward_calc(double dist, double d0, bool col, bool goal) {
  const double r_g = goal ? 1.0 : 0.05 * (d0 - dist);
  const double r_c = col ? -1.0 : 0.0;
  return (r_g + r_c) + (-0.05);
}

}  // namespace ffmp
