// voxnav_env.hip -- MI355X (gfx950) batched voxel-grid exploration env.
//
// The hot path of Noimps/3D-Navigation-Reinforcement-Learning is
// GridAgent.step/reset in envs/CubicEnv.py, run one agent per OS process
// under SB3's SubprocVecEnv (train/Grid_Train.py:191-192).  Here every agent
// is one lane of a 64-wide wavefront and a launch advances all N agents by
// K steps.  See DESIGN.md for the data layout and the roofline.
//
// Layout in HBM
//   hot state   uint4 per agent (16 B, SoA across agents -> coalesced)
//     w0 = x | y<<8 | z<<16 | facing<<21 | last_action<<23 | done<<26
//          | last_bump<<27 | near_wall<<28 | was_near_wall<<29
//     w1 = step_count (24 b, saturating) | cells_insight_down<<24
//     w2 = visited_count (24 b) | room<<24
//     w3 = bump_count (26 b, saturating) | move_mask<<26  (6 b: first cell
//          free in +x,-x,+y,-y,+z,-z -> the next move needs no memory read)
//   belief map  int8 per cell (the reference's internal_grid; -2 wall,
//     -1 unknown, 0 known free, n visits saturating at 127 -- the obs clips
//     at 20 (CubicEnv.py:274) and the reward caps at 25 (:180), so the
//     saturation is observationally exact).  Per agent the map is bricked:
//     4x4 (x,y) columns of PH bytes (z contiguous), bricks x-major, so the
//     4x4x4 window is <=4 bricks and an x/y ray crosses <=4 bricks.
//   room tables (tiny, L2 resident): per cell an 8-byte ray record with the
//     free-run length to the first wall/OOB in each of the 6 axis directions
//     (bit7 = ended at a wall) and a wall flag, so a sensing sweep needs one
//     8-byte load instead of 6L grid probes.
//
// Arithmetic follows the reference bit for bit: reward in f64 in the
// reference's operation order (file compiled with -ffp-contract=off), obs
// window values from a 23-entry f32 table built on the host with IEEE f32
// division, obs[68], [71], [72] as f64 quotients rounded to f32.

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <new>
#include <string>
#include <vector>

#include "voxnav.h"

namespace {

// ----------------------------------------------------------------------------
// errors
// ----------------------------------------------------------------------------
thread_local std::string g_last_error;

int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof(buf), fmt, ap);
    va_end(ap);
    g_last_error = buf;
    return code;
}

#define VN_HIP(expr)                                                                        \
    do {                                                                                    \
        hipError_t e_ = (expr);                                                             \
        if (e_ != hipSuccess) return fail(VN_ERR_HIP, "%s: %s", #expr, hipGetErrorString(e_)); \
    } while (0)

constexpr int MT_N = 624;
constexpr int MT_C = 8;  // MT words captured by the streaming seed (draws 0..7)

// init_genrand(19650218): the seed-independent prefix of CPython's
// init_by_array (Modules/_randommodule.c); filled once per device.
__constant__ uint32_t c_mt_g[MT_N];

// ----------------------------------------------------------------------------
// device data structures
// ----------------------------------------------------------------------------
struct RoomDesc {          // 32 B, two uint4
    uint32_t whd;          // W | D<<8 | H<<16
    uint32_t total_free;   // interior free cells = max_steps (CubicEnv.py:450-459)
    uint32_t ray_off;      // first ray record of the room
    uint32_t start_off;    // first packed start cell (x | y<<8 | z<<16)
    int32_t fixed_start;   // packed "Start position" or -1
    uint32_t bricks;       // ceil(W/4) | ceil(D/4)<<16
    uint32_t pad0, pad1;
};

struct Room {
    int W, D, H;
    uint32_t total_free, ray_off, start_off;
    int32_t fixed_start;
    int nbx, nby;
};

struct Agent {
    int x, y, z, facing, last_action;
    bool done, last_bump, near_wall, was_near_wall;
    uint32_t step_count, visited, bumps, move_mask;
    int cid, room;
};

struct Params {
    uint4 *hot;
    uint32_t *next_seed;
    int8_t *belief;
    const uint4 *rooms;
    const uint2 *rays;
    const uint32_t *starts;
    const float *lut;
    int32_t *err;
    int N, L, nby, ph;
    uint32_t map_bytes;
    int n_rooms, use_room_draw, autoreset;
    uint32_t seed_stride;
    double crash_penalty, finish;
    uint64_t gid_base;
    // per call
    int K;
    const int32_t *actions;  // NULL -> Philox random policy
    uint64_t policy_seed, t0;
    int32_t *actions_out;
    float *obs, *reward, *terminal_obs;
    double *reward64;
    uint8_t *term, *trunc;
    const int64_t *seeds;    // reset-only launches
    const uint8_t *mask;
};

__device__ __forceinline__ Agent unpack(uint4 s) {
    Agent g;
    g.x = s.x & 0xff;
    g.y = (s.x >> 8) & 0xff;
    g.z = (s.x >> 16) & 0x1f;
    g.facing = (s.x >> 21) & 3;
    g.last_action = (s.x >> 23) & 7;
    g.done = (s.x >> 26) & 1;
    g.last_bump = (s.x >> 27) & 1;
    g.near_wall = (s.x >> 28) & 1;
    g.was_near_wall = (s.x >> 29) & 1;
    g.step_count = s.y & 0xffffffu;
    g.cid = s.y >> 24;
    g.visited = s.z & 0xffffffu;
    g.room = s.z >> 24;
    g.bumps = s.w & 0x3ffffffu;
    g.move_mask = s.w >> 26;
    return g;
}

__device__ __forceinline__ uint4 pack(const Agent &g) {
    uint4 s;
    s.x = (uint32_t)g.x | ((uint32_t)g.y << 8) | ((uint32_t)g.z << 16) | ((uint32_t)g.facing << 21) |
          ((uint32_t)g.last_action << 23) | ((uint32_t)g.done << 26) | ((uint32_t)g.last_bump << 27) |
          ((uint32_t)g.near_wall << 28) | ((uint32_t)g.was_near_wall << 29);
    s.y = g.step_count | ((uint32_t)g.cid << 24);
    s.z = g.visited | ((uint32_t)g.room << 24);
    s.w = g.bumps | (g.move_mask << 26);
    return s;
}

__device__ __forceinline__ Room load_room(const Params &p, int r) {
    const uint4 a = p.rooms[2 * r];
    const uint4 b = p.rooms[2 * r + 1];
    Room R;
    R.W = a.x & 0xff;
    R.D = (a.x >> 8) & 0xff;
    R.H = (a.x >> 16) & 0xff;
    R.total_free = a.y;
    R.ray_off = a.z;
    R.start_off = a.w;
    R.fixed_start = (int32_t)b.x;
    R.nbx = b.y & 0xffff;
    R.nby = b.y >> 16;
    return R;
}

// byte offset of cell (x,y,z) inside one agent's bricked belief map
__device__ __forceinline__ uint32_t boff(int x, int y, int z, int nby, int ph) {
    return (uint32_t)((((((x >> 2) * nby + (y >> 2)) << 4) + ((x & 3) << 2) + (y & 3)) * ph) + z);
}

// ----------------------------------------------------------------------------
// CPython random: streaming MT19937 seed (init_by_array with a one-word key)
// that keeps only the words the first MT_C outputs need, so a reset runs
// from registers without a 2.5 KB state array.
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= (y >> 11);
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= (y >> 18);
    return y;
}

__device__ __forceinline__ uint32_t mix1(uint32_t g, uint32_t p, uint32_t seed) {
    return (g ^ ((p ^ (p >> 30)) * 1664525u)) + seed;
}
__device__ __forceinline__ uint32_t mix2(uint32_t m, uint32_t q, uint32_t i) {
    return (m ^ ((q ^ (q >> 30)) * 1566083941u)) - i;
}

// First MT_C outputs of random.seed(seed) -> out[0..MT_C-1].
__device__ void mt_first_outputs(uint32_t seed, uint32_t out[MT_C]) {
    // init_by_array loop 1, i = 1..623 (key[j] + j == seed for a one-word key)
    uint32_t p = mix1(c_mt_g[1], c_mt_g[0], seed);
    const uint32_t m1_1 = p;
    for (int i = 2; i < MT_N; ++i) p = mix1(c_mt_g[i], p, seed);
    const uint32_t m1b1 = mix1(m1_1, p, seed);  // wrap: i = 1 again, mt[0] = mt[623]
    // loop 2, i = 2..623, recomputing loop-1 words on the fly
    uint32_t p1 = m1_1, q = m1b1;
    uint32_t lo[MT_C + 1], hi[MT_C];
#pragma unroll
    for (int i = 2; i <= MT_C; ++i) {
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
        lo[i] = q;
    }
    for (int i = MT_C + 1; i < 397; ++i) {
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
    }
#pragma unroll
    for (int i = 397; i < 397 + MT_C; ++i) {
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
        hi[i - 397] = q;
    }
    for (int i = 397 + MT_C; i < MT_N; ++i) {
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
    }
    lo[1] = mix2(m1b1, q, 1u);
    lo[0] = 0x80000000u;
#pragma unroll
    for (int j = 0; j < MT_C; ++j) {
        const uint32_t y = (lo[j] & 0x80000000u) | (lo[j + 1] & 0x7fffffffu);
        out[j] = mt_temper(hi[j] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
    }
}

// Final (pre-twist) state word F[idx] of random.seed(seed); slow path.
__device__ __noinline__ uint32_t mt_state_word(uint32_t seed, int idx) {
    if (idx == 0) return 0x80000000u;
    uint32_t p = mix1(c_mt_g[1], c_mt_g[0], seed);
    const uint32_t m1_1 = p;
    for (int i = 2; i < MT_N; ++i) p = mix1(c_mt_g[i], p, seed);
    const uint32_t m1b1 = mix1(m1_1, p, seed);
    uint32_t p1 = m1_1, q = m1b1, cap = 0;
    for (int i = 2; i < MT_N; ++i) {
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
        if (i == idx) cap = q;
    }
    return idx == 1 ? mix2(m1b1, q, 1u) : cap;
}

// Output j (>= MT_C) of the first twist; valid for j < 227.
__device__ __noinline__ uint32_t mt_output_slow(uint32_t seed, int j, int32_t *err) {
    if (j >= MT_N - 397) {
        atomicOr(err, 1);
        return 0u;
    }
    const uint32_t y = (mt_state_word(seed, j) & 0x80000000u) | (mt_state_word(seed, j + 1) & 0x7fffffffu);
    return mt_temper(mt_state_word(seed, j + 397) ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
}

struct MtStream {
    uint32_t seed;
    uint32_t buf[MT_C];
    int used;
    int32_t *err;

    __device__ uint32_t next() {
        uint32_t r;
        if (used < MT_C) {
            r = buf[0];
#pragma unroll
            for (int t = 0; t < MT_C - 1; ++t) buf[t] = buf[t + 1];
        } else {
            r = mt_output_slow(seed, used, err);
        }
        ++used;
        return r;
    }
    // random._randbelow_with_getrandbits(n), n >= 1
    __device__ uint32_t below(uint32_t n) {
        const int k = 32 - __clz(n);
        uint32_t r = next() >> (32 - k);
        while (r >= n) r = next() >> (32 - k);
        return r;
    }
};

// ----------------------------------------------------------------------------
// Philox4x32-10 random policy (build-defined)
// ----------------------------------------------------------------------------
__device__ __forceinline__ int philox_action(uint64_t key, uint64_t gid, uint64_t t) {
    uint32_t c0 = (uint32_t)gid, c1 = (uint32_t)(gid >> 32), c2 = (uint32_t)t, c3 = (uint32_t)(t >> 32);
    uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k0 += 0x9E3779B9u;
            k1 += 0xBB67AE85u;
        }
        const uint32_t lo0 = 0xD2511F53u * c0, hi0 = __umulhi(0xD2511F53u, c0);
        const uint32_t lo1 = 0xCD9E8D57u * c2, hi1 = __umulhi(0xCD9E8D57u, c2);
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
    }
    return (int)(((uint64_t)c0 * 6u) >> 32);
}

// ----------------------------------------------------------------------------
// sensing + observation (get_obs, envs/CubicEnv.py:254-312, with the ray
// side effects of _sense_direction :345-397 and the visit update of
// _mark_visited/do_action :156-166 folded into the same belief pass)
// ----------------------------------------------------------------------------
// ray directions: 0 +x, 1 -x, 2 +y, 3 -y, 4 +z (up), 5 -z (down)

__device__ __forceinline__ uint32_t patch_byte(uint32_t b, int s, int nf, bool wh) {
    if (s <= nf) return b == 0xffu ? 0u : b;       // known free: -1 -> 0  (:386-387)
    if (wh && s == nf + 1) return 0xfeu;            // first wall -> -2     (:374-375)
    return b;
}

// Destination of the observation row.  With auto-reset, a step that ends the
// episode writes its obs to the terminal row (NULL: dropped) and the reset
// obs goes to the regular row; `ends` needs the post-move visited count.
struct ObsDst {
    float *row;
    float *term_row;
    bool select;       // auto-reset step: choose between row and term_row
    bool truncated;
};

template <int LMAX, bool FRESH>
__device__ __forceinline__ int sense_observe(const Params &p, int8_t *map, Agent &g, const Room &R, bool moved,
                                             bool &explored, const float *lut, ObsDst dst) {
    const int x = g.x, y = g.y, z = g.z, nby = p.nby, ph = p.ph, L = p.L;
    const uint2 rec = p.rays[R.ray_off + (uint32_t)((x * R.D + y) * R.H + z)];

    // ---- 4x4x4 window, one funnel-shifted dword pair per (x,y) column ----
    uint32_t win[16];
    if (FRESH) {
#pragma unroll
        for (int c = 0; c < 16; ++c) win[c] = 0xffffffffu;
    } else {
        const int d0 = (z - 2) >> 2;
        const int sh = ((z - 2) & 3) * 8;
        const int ndw = ph >> 2;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int cx = x + i - 2, cy = y + j - 2;
                uint32_t lo = 0xffffffffu, hi = 0xffffffffu;
                if (cx >= 0 && cx < R.W && cy >= 0 && cy < R.D) {
                    const uint32_t *col = reinterpret_cast<const uint32_t *>(map + boff(cx, cy, 0, nby, ph));
                    if (d0 >= 0) lo = col[d0];
                    if (d0 + 1 < ndw) hi = col[d0 + 1];
                }
                win[i * 4 + j] = (uint32_t)(((((uint64_t)hi) << 32) | lo) >> sh);
            }
        }
    }

    // ---- ray extents ----
    int nf[6];
    bool wh[6];
    bool near = false;
    int center;
    uint32_t mm = 0;
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const uint32_t e = (r < 4 ? (rec.x >> (8 * r)) : (rec.y >> (8 * (r - 4)))) & 0xffu;
        const int n = (int)(e & 0x7fu);
        const bool wf = (e >> 7) != 0;
        nf[r] = n < L ? n : L;
        wh[r] = wf && n < L;
        near |= (n == 0) && wf;   // wall at step 1 -> near_wall (:378-379)
        mm |= (n > 0 ? 1u : 0u) << r;
    }

    // ---- ray cells outside the window: load (all first), patch, store ----
    // in-window steps: +x,+y,+z s=1; -x,-y,-z s=1,2
    constexpr int NS = LMAX;  // slots s = 0..LMAX-1 map to steps s0+slot
    uint32_t rv[6][NS];
    const uint32_t cb = boff(x, y, 0, nby, ph);
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const int s0 = (r & 1) ? 3 : 2;
        const int lim = nf[r] + (wh[r] ? 1 : 0);
#pragma unroll
        for (int t = 0; t < NS; ++t) {
            const int s = s0 + t;
            rv[r][t] = 0xffu;
            if (!FRESH && s <= LMAX && s <= lim) {
                uint32_t a;
                switch (r) {
                    case 0: a = boff(x + s, y, z, nby, ph); break;
                    case 1: a = boff(x - s, y, z, nby, ph); break;
                    case 2: a = boff(x, y + s, z, nby, ph); break;
                    case 3: a = boff(x, y - s, z, nby, ph); break;
                    case 4: a = cb + z + s; break;
                    default: a = cb + z - s; break;
                }
                rv[r][t] = (uint8_t)map[a];
            }
        }
    }
#pragma unroll
    for (int r = 0; r < 6; ++r) {
        const int s0 = (r & 1) ? 3 : 2;
        const int lim = nf[r] + (wh[r] ? 1 : 0);
#pragma unroll
        for (int t = 0; t < NS; ++t) {
            const int s = s0 + t;
            if (s <= LMAX && s <= lim) {
                const uint32_t nb = patch_byte(rv[r][t], s, nf[r], wh[r]);
                if (nb != rv[r][t]) {
                    uint32_t a;
                    switch (r) {
                        case 0: a = boff(x + s, y, z, nby, ph); break;
                        case 1: a = boff(x - s, y, z, nby, ph); break;
                        case 2: a = boff(x, y + s, z, nby, ph); break;
                        case 3: a = boff(x, y - s, z, nby, ph); break;
                        case 4: a = cb + z + s; break;
                        default: a = cb + z - s; break;
                    }
                    map[a] = (int8_t)nb;
                }
            }
        }
    }

    // ---- center cell: _mark_visited(target) then the +1 of :165-166 ----
    {
        int t;
        if (FRESH) {
            t = 1;                                    // start cell (:85)
        } else {
            t = (int)(int8_t)((win[10] >> 16) & 0xffu);
            if (moved) {
                if (t == 0) {
                    t = 1;
                    ++g.visited;
                    explored = true;
                } else if (t > 0) {
                    t += 1;
                }
            }
            t += 1;
            if (t > 127) t = 127;
        }
        win[10] = (win[10] & 0xff00ffffu) | ((uint32_t)(t & 0xff) << 16);
        map[cb + z] = (int8_t)t;
        center = t;
    }

    // ---- in-window ray cells: patch + store ----
    // (column index c = (dx+2)*4 + (dy+2), byte = dz+2)
    auto patch_win = [&](int c, int byte, int r, int s) {
        const uint32_t b = (win[c] >> (8 * byte)) & 0xffu;
        if (s <= nf[r] || (wh[r] && s == nf[r] + 1)) {
            const uint32_t nb = patch_byte(b, s, nf[r], wh[r]);
            if (nb != b) {
                win[c] = (win[c] & ~(0xffu << (8 * byte))) | (nb << (8 * byte));
                uint32_t a;
                switch (r) {
                    case 0: a = boff(x + s, y, z, nby, ph); break;
                    case 1: a = boff(x - s, y, z, nby, ph); break;
                    case 2: a = boff(x, y + s, z, nby, ph); break;
                    case 3: a = boff(x, y - s, z, nby, ph); break;
                    case 4: a = cb + z + s; break;
                    default: a = cb + z - s; break;
                }
                map[a] = (int8_t)nb;
            }
        }
    };
    patch_win(14, 2, 0, 1);
    patch_win(6, 2, 1, 1);
    patch_win(2, 2, 1, 2);
    patch_win(11, 2, 2, 1);
    patch_win(9, 2, 3, 1);
    patch_win(8, 2, 3, 2);
    patch_win(10, 3, 4, 1);
    patch_win(10, 1, 5, 1);
    patch_win(10, 0, 5, 2);

    g.near_wall = g.near_wall || near;
    g.cid = nf[5];
    g.move_mask = mm;

    // ---- observation row (80 f32, 20 x 16-B stores) ----
    float *obs_row = dst.row;
    if (dst.select &&
        (dst.truncated || g.done || (double)g.visited / (double)R.total_free >= p.finish))
        obs_row = dst.term_row;
    if (obs_row) {
        float4 *o4 = reinterpret_cast<float4 *>(obs_row);
#pragma unroll
        for (int c = 0; c < 16; ++c) {
            float v[4];
#pragma unroll
            for (int b = 0; b < 4; ++b) {
                int cv = (int)(int8_t)((win[c] >> (8 * b)) & 0xffu);
                cv = (cv > 20 ? 20 : cv) + 2;           // clip(-2, 20) + 2   (:274-275)
                v[b] = lut[cv];
            }
            o4[c] = make_float4(v[0], v[1], v[2], v[3]);
        }
        float t[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) t[k] = 0.0f;
#pragma unroll
        for (int k = 0; k < 4; ++k) t[k] = (g.facing == k) ? 1.0f : 0.0f;   // (:279-280)
        t[4] = (float)((double)g.last_action / 5.0);                   // (:284)
        t[5] = g.was_near_wall ? 1.0f : 0.0f;                          // (:285)
        t[6] = g.last_bump ? 1.0f : 0.0f;                              // (:286)
        t[7] = (float)((double)g.cid / (double)L);                     // (:287)
        t[8] = (float)((double)g.visited / (double)R.total_free);      // (:291)
#pragma unroll
        for (int c = 0; c < 4; ++c) o4[16 + c] = make_float4(t[4 * c], t[4 * c + 1], t[4 * c + 2], t[4 * c + 3]);
    }
    return center;
}

// ----------------------------------------------------------------------------
// reset (envs/CubicEnv.py:77-108): draws for lanes with `need`, then the
// whole wave clears each resetting agent's bricks (1 KiB per instruction),
// then each resetting lane senses from its start cell.
// ----------------------------------------------------------------------------
template <int LMAX>
__device__ __forceinline__ void wave_reset(const Params &p, int8_t *belief_base, int agent, bool need, uint32_t seed,
                                           Agent &g, Room &R, const float *lut, float *obs_row) {
    if (need) {
        MtStream mt;
        mt.seed = seed;
        mt.used = 0;
        mt.err = p.err;
        mt_first_outputs(seed, mt.buf);
        const int room = p.use_room_draw ? (int)mt.below((uint32_t)p.n_rooms) : 0;   // :407
        R = load_room(p, room);
        int sx, sy, sz;
        if (R.fixed_start >= 0) {
            sx = R.fixed_start & 0xff;
            sy = (R.fixed_start >> 8) & 0xff;
            sz = (R.fixed_start >> 16) & 0xff;
        } else {
            const uint32_t s = p.starts[R.start_off + mt.below(R.total_free)];      // :462
            sx = s & 0xff;
            sy = (s >> 8) & 0xff;
            sz = (s >> 16) & 0xff;
        }
        const uint2 rec = p.rays[R.ray_off + (uint32_t)((sx * R.D + sy) * R.H + sz)];
        if ((rec.y >> 16) & 1u) {                                                   // :464-466
            const uint32_t s = p.starts[R.start_off + mt.below(R.total_free)];
            sx = s & 0xff;
            sy = (s >> 8) & 0xff;
            sz = (s >> 16) & 0xff;
        }
        g.room = room;
        g.x = sx;
        g.y = sy;
        g.z = sz;
        g.facing = 0;
        g.last_action = 0;
        g.done = g.last_bump = g.near_wall = g.was_near_wall = false;
        g.step_count = 0;
        g.visited = 1;
        g.bumps = 0;
        g.cid = 0;
        g.move_mask = 0;
    }
    // cooperative clear of the new room's bricks to -1 (0xff)
    uint64_t m = __ballot(need);
    const int lane = threadIdx.x & 63;
    const uint32_t brick16 = (uint32_t)p.ph;  // 16-byte chunks per brick
    while (m) {
        const int l = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const int a = __shfl(agent, l);
        const int nbx = __shfl(R.nbx, l);
        const int nbyr = __shfl(R.nby, l);
        uint4 *base = reinterpret_cast<uint4 *>(belief_base + (size_t)a * p.map_bytes);
        const uint32_t total = (uint32_t)(nbx * nbyr) * brick16;
        for (uint32_t c = lane; c < total; c += 64) {
            const uint32_t brick = c / brick16, w = c - brick * brick16;
            const uint32_t bx = brick / (uint32_t)nbyr, by = brick - bx * (uint32_t)nbyr;
            base[(bx * (uint32_t)p.nby + by) * brick16 + w] = make_uint4(~0u, ~0u, ~0u, ~0u);
        }
        (void)nbx;
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (need) {
        bool explored = false;
        sense_observe<LMAX, true>(p, belief_base + (size_t)agent * p.map_bytes, g, R, false, explored, lut,
                                  ObsDst{obs_row, nullptr, false, false});
    }
}

// ----------------------------------------------------------------------------
// the step kernel: one lane per agent, K fused steps, SB3 auto-reset
// ----------------------------------------------------------------------------
template <int LMAX, bool RESET_ONLY>
__global__ __launch_bounds__(256) void env_kernel(Params p) {
    __shared__ float lut[32];
    if (threadIdx.x < 32) lut[threadIdx.x] = p.lut[threadIdx.x];
    __syncthreads();

    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const bool active = i < p.N;
    const int ai = active ? i : 0;
    Agent g = unpack(p.hot[ai]);
    Room R = load_room(p, active ? g.room : 0);
    uint32_t next_seed = p.next_seed[ai];
    int8_t *map = p.belief + (size_t)ai * p.map_bytes;

    if (RESET_ONLY) {
        const bool need = active && (p.mask == nullptr || p.mask[i] != 0);
        const uint32_t seed = need ? (uint32_t)p.seeds[i] : 0u;
        wave_reset<LMAX>(p, p.belief, ai, need, seed, g, R, lut, need ? p.obs + (size_t)i * VN_OBS_DIM : nullptr);
        if (need) {
            p.hot[i] = pack(g);
            p.next_seed[i] = seed + p.seed_stride;
        }
        return;
    }

    for (int k = 0; k < p.K; ++k) {
        bool finished = false;
        const size_t row = (size_t)k * (size_t)p.N + (size_t)i;
        if (active) {
            const int a = p.actions ? p.actions[row]
                                    : philox_action(p.policy_seed, p.gid_base + (uint64_t)i, p.t0 + (uint64_t)k);
            if (p.actions_out) p.actions_out[row] = a;

            // step() prologue (:111-116)
            if (g.near_wall) {
                g.was_near_wall = true;
                g.near_wall = false;
            }
            if (g.step_count < 0xffffffu) ++g.step_count;
            const bool truncated = g.step_count >= R.total_free;

            // do_action (:134-166): relative move table by facing -> axis dir
            int dir;
            if (a < 4) {
                // rows: fwd, right, back, left; cols: facing N,E,S,W
                // dirs 0 +x, 1 -x, 2 +y, 3 -y
                constexpr uint32_t kDir = (2u << 0) | (0u << 2) | (3u << 4) | (1u << 6)      // fwd
                                          | (0u << 8) | (3u << 10) | (1u << 12) | (2u << 14)  // right
                                          | (3u << 16) | (1u << 18) | (2u << 20) | (0u << 22)  // back
                                          | (1u << 24) | (2u << 26) | (0u << 28) | (3u << 30); // left
                dir = (int)((kDir >> (2 * (a * 4 + g.facing))) & 3u);
                g.facing = (int)((0x8Du >> (2 * dir)) & 3u);  // +x->E(1) -x->W(3) +y->N(0) -y->S(2)
            } else {
                dir = (a == 4) ? 4 : 5;
            }
            const bool moved = (g.move_mask >> dir) & 1u;
            if (moved) {
                g.x += (dir == 0) - (dir == 1);
                g.y += (dir == 2) - (dir == 3);
                g.z += (dir == 4) - (dir == 5);
            }

            bool explored = false;
            const ObsDst dst{p.obs + row * VN_OBS_DIM,
                             p.terminal_obs ? p.terminal_obs + row * VN_OBS_DIM : nullptr,
                             p.autoreset != 0, truncated};
            const int vv = sense_observe<LMAX, false>(p, map, g, R, moved, explored, lut, dst);

            // compute_reward (:169-224), f64 in the reference's order
            double r = -0.05;
            const double pen = (double)vv * 0.02;
            r -= (0.5 < pen) ? 0.5 : pen;
            const bool bumped = !moved;
            if (bumped) {
                g.last_bump = true;
                if (g.bumps < 0x3ffffffu) ++g.bumps;
                r += p.crash_penalty;
            } else {
                g.last_bump = false;
                if (g.was_near_wall) {
                    g.was_near_wall = false;
                    r += 0.15;
                }
                if (g.last_action != 2 && a == g.last_action && g.last_action < 4) r += 0.05;
                if (g.last_action == 2 && a == 2) r -= 0.5;
            }
            if (explored) r += 1.0;
            const double pct2 = (double)g.visited / (double)R.total_free;
            if (pct2 >= p.finish) {
                g.done = true;
                r += 100.0;
            }
            if (truncated) r += -5.0;
            g.last_action = a;

            if (p.reward) p.reward[row] = (float)r;
            if (p.reward64) p.reward64[row] = r;
            if (p.term) p.term[row] = g.done ? 1 : 0;
            if (p.trunc) p.trunc[row] = truncated ? 1 : 0;
            finished = g.done || truncated;
        }
        const bool need = p.autoreset && finished;
        if (__ballot(need)) {
            const uint32_t seed = next_seed;
            wave_reset<LMAX>(p, p.belief, ai, need, seed, g, R, lut,
                             need ? p.obs + row * VN_OBS_DIM : nullptr);
            if (need) next_seed = seed + p.seed_stride;
        }
    }
    if (active) {
        p.hot[i] = pack(g);
        p.next_seed[i] = next_seed;
    }
}

// ----------------------------------------------------------------------------
// exports (parity dumps)
// ----------------------------------------------------------------------------
__global__ void export_state_kernel(Params p, int64_t *out) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.N) return;
    const Agent g = unpack(p.hot[i]);
    const Room R = load_room(p, g.room);
    int64_t *o = out + (size_t)i * VN_STATE_FIELDS;
    o[0] = g.x; o[1] = g.y; o[2] = g.z; o[3] = g.facing; o[4] = g.last_action;
    o[5] = g.step_count; o[6] = g.visited; o[7] = g.bumps;
    o[8] = g.done; o[9] = g.last_bump; o[10] = g.near_wall; o[11] = g.was_near_wall;
    o[12] = g.cid; o[13] = g.room; o[14] = R.total_free; o[15] = p.next_seed[i];
}

__global__ void export_belief_kernel(Params p, int8_t *out, int pw, int pd) {
    const size_t cells = (size_t)pw * pd * p.ph;
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= cells * (size_t)p.N) return;
    const int i = (int)(gid / cells);
    const size_t c = gid - (size_t)i * cells;
    const int z = (int)(c % p.ph), y = (int)((c / p.ph) % pd), x = (int)(c / ((size_t)p.ph * pd));
    const Agent g = unpack(p.hot[i]);
    const Room R = load_room(p, g.room);
    int8_t v = -128;
    if (x < R.W && y < R.D && z < R.H) v = p.belief[(size_t)i * p.map_bytes + boff(x, y, z, p.nby, p.ph)];
    out[gid] = v;
}

// ----------------------------------------------------------------------------
// GAE (SB3 RolloutBuffer.compute_returns_and_advantage), one lane per env,
// reverse scan over T; f32 in numpy's evaluation order, no contraction.
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gae_kernel(const float *__restrict__ rew, const float *__restrict__ val,
                                                  const float *__restrict__ starts, const float *__restrict__ last_v,
                                                  const float *__restrict__ dones, int T, int N, float g32, float gl32,
                                                  float *__restrict__ adv, float *__restrict__ ret) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    float last = 0.0f;
    float nv = last_v[i];
    float nnt = 1.0f - dones[i];
    for (int t = T - 1; t >= 0; --t) {
        const size_t o = (size_t)t * N + i;
        const float v = val[o];
        const float r = rew[o];
        const float s = (t > 0) ? starts[o] : 0.0f;  // episode_starts[t] feeds step t-1
        const float gv = g32 * nv;
        const float gvn = gv * nnt;
        const float sum = r + gvn;
        const float delta = sum - v;
        const float glnn = gl32 * nnt;
        const float carry = glnn * last;
        last = delta + carry;
        adv[o] = last;
        ret[o] = last + v;
        nv = v;
        nnt = 1.0f - s;
    }
}

}  // namespace

// ============================================================================
// host side
// ============================================================================
struct VnEnv {
    int device = 0;
    int N = 0;
    VnConfig cfg{};
    int n_rooms = 0;
    int pw = 0, pd = 0, ph = 0, nbx = 0, nby = 0;
    uint32_t map_bytes = 0;
    size_t device_bytes = 0;
    std::vector<uint32_t> total_free;
    uint4 *d_rooms = nullptr;
    uint2 *d_rays = nullptr;
    uint32_t *d_starts = nullptr;
    float *d_lut = nullptr;
    uint4 *d_hot = nullptr;
    uint32_t *d_seed = nullptr;
    int8_t *d_belief = nullptr;
    int32_t *d_err = nullptr;
};

namespace {

bool g_mt_ready[64] = {false};

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev) {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) (void)hipSetDevice(dev);
    }
    ~DeviceGuard() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

int ensure_mt_table(int device) {
    if (device < 0 || device >= 64) return fail(VN_ERR_INVALID, "device %d out of range", device);
    if (g_mt_ready[device]) return VN_OK;
    uint32_t g[MT_N];
    g[0] = 19650218u;
    for (int i = 1; i < MT_N; ++i) g[i] = 1812433253u * (g[i - 1] ^ (g[i - 1] >> 30)) + (uint32_t)i;
    VN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(c_mt_g), g, sizeof(g)));
    g_mt_ready[device] = true;
    return VN_OK;
}

Params base_params(VnEnv *e) {
    Params p;
    std::memset(&p, 0, sizeof(p));
    p.hot = e->d_hot;
    p.next_seed = e->d_seed;
    p.belief = e->d_belief;
    p.rooms = e->d_rooms;
    p.rays = e->d_rays;
    p.starts = e->d_starts;
    p.lut = e->d_lut;
    p.err = e->d_err;
    p.N = e->N;
    p.L = e->cfg.local_map_length;
    p.nby = e->nby;
    p.ph = e->ph;
    p.map_bytes = e->map_bytes;
    p.n_rooms = e->n_rooms;
    p.use_room_draw = e->cfg.use_room_draw;
    p.autoreset = e->cfg.autoreset;
    p.seed_stride = (uint32_t)(uint64_t)e->cfg.seed_stride;
    p.crash_penalty = e->cfg.crash_penalty;
    p.finish = e->cfg.finish_percentage;
    p.gid_base = (uint64_t)e->cfg.agent_id_base;
    p.K = 1;
    return p;
}

template <bool RESET_ONLY>
int launch_env(VnEnv *e, const Params &p, hipStream_t s) {
    const dim3 block(256);
    const dim3 grid((unsigned)((e->N + 255) / 256));
    const int L = e->cfg.local_map_length;
    if (L <= 4)
        hipLaunchKernelGGL((env_kernel<4, RESET_ONLY>), grid, block, 0, s, p);
    else if (L <= 8)
        hipLaunchKernelGGL((env_kernel<8, RESET_ONLY>), grid, block, 0, s, p);
    else if (L <= 12)
        hipLaunchKernelGGL((env_kernel<12, RESET_ONLY>), grid, block, 0, s, p);
    else
        hipLaunchKernelGGL((env_kernel<16, RESET_ONLY>), grid, block, 0, s, p);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

void free_env(VnEnv *e) {
    if (!e) return;
    (void)hipFree(e->d_rooms);
    (void)hipFree(e->d_rays);
    (void)hipFree(e->d_starts);
    (void)hipFree(e->d_lut);
    (void)hipFree(e->d_hot);
    (void)hipFree(e->d_seed);
    (void)hipFree(e->d_belief);
    (void)hipFree(e->d_err);
    delete e;
}

}  // namespace

extern "C" {

const char *vn_last_error(void) { return g_last_error.c_str(); }

int vn_abi_version(void) { return VN_ABI_VERSION; }

int vn_create(const VnRoomSet *rooms, int32_t n_agents, const VnConfig *cfg, int32_t device, VnEnv **out) {
    if (!rooms || !cfg || !out) return fail(VN_ERR_INVALID, "NULL argument");
    *out = nullptr;
    if (n_agents <= 0) return fail(VN_ERR_INVALID, "n_agents must be > 0 (got %d)", n_agents);
    if (rooms->n_rooms <= 0 || rooms->n_rooms > VN_MAX_ROOMS)
        return fail(VN_ERR_INVALID, "n_rooms must be in 1..%d (got %d)", VN_MAX_ROOMS, rooms->n_rooms);
    if (!rooms->whd || !rooms->walls) return fail(VN_ERR_INVALID, "rooms->whd / rooms->walls is NULL");
    if (cfg->local_map_length < 1 || cfg->local_map_length > VN_MAX_L)
        return fail(VN_ERR_INVALID, "local_map_length must be in 1..%d (got %d)", VN_MAX_L, cfg->local_map_length);

    // ---- rooms -> descriptors, ray records, start lists ----
    const int nr = rooms->n_rooms;
    std::vector<uint32_t> desc((size_t)nr * 8, 0);
    std::vector<uint2> rays;
    std::vector<uint32_t> starts;
    std::vector<uint32_t> total_free(nr);
    int maxW = 0, maxD = 0, maxH = 0;
    size_t woff = 0;
    for (int r = 0; r < nr; ++r) {
        const int W = rooms->whd[3 * r], D = rooms->whd[3 * r + 1], H = rooms->whd[3 * r + 2];
        if (W < 1 || W > VN_MAX_W || D < 1 || D > VN_MAX_D || H < 1 || H > VN_MAX_H)
            return fail(VN_ERR_ROOM, "room %d: size %dx%dx%d outside 1..%d x 1..%d x 1..%d", r, W, D, H, VN_MAX_W,
                        VN_MAX_D, VN_MAX_H);
        const uint8_t *wall = rooms->walls + woff;
        auto is_wall = [&](int x, int y, int z) { return wall[((size_t)x * D + y) * H + z] != 0; };
        const uint32_t ray_off = (uint32_t)rays.size(), start_off = (uint32_t)starts.size();
        // interior scan in x -> y -> z order (envs/CubicEnv.py:450-457)
        uint32_t tf = 0;
        for (int x = 1; x < W - 1; ++x)
            for (int y = 1; y < D - 1; ++y)
                for (int z = 1; z < H - 1; ++z)
                    if (!is_wall(x, y, z)) {
                        starts.push_back((uint32_t)x | ((uint32_t)y << 8) | ((uint32_t)z << 16));
                        ++tf;
                    }
        if (tf == 0) return fail(VN_ERR_ROOM, "room %d has no interior free cell (random.choice of [])", r);
        total_free[r] = tf;
        // ray records
        static const int DX[6] = {1, -1, 0, 0, 0, 0}, DY[6] = {0, 0, 1, -1, 0, 0}, DZ[6] = {0, 0, 0, 0, 1, -1};
        for (int x = 0; x < W; ++x)
            for (int y = 0; y < D; ++y)
                for (int z = 0; z < H; ++z) {
                    uint32_t e8[8] = {0, 0, 0, 0, 0, 0, 0, 0};
                    for (int d = 0; d < 6; ++d) {
                        int n = 0;
                        uint32_t wf = 0;
                        for (int s = 1;; ++s) {
                            const int nx = x + DX[d] * s, ny = y + DY[d] * s, nz = z + DZ[d] * s;
                            if (nx < 0 || nx >= W || ny < 0 || ny >= D || nz < 0 || nz >= H) break;
                            if (is_wall(nx, ny, nz)) {
                                wf = 1;
                                break;
                            }
                            ++n;
                        }
                        if (n > 127) {
                            n = 127;
                            wf = 0;
                        }
                        e8[d] = (uint32_t)n | (wf << 7);
                    }
                    e8[6] = is_wall(x, y, z) ? 1u : 0u;
                    uint2 rec;
                    rec.x = e8[0] | (e8[1] << 8) | (e8[2] << 16) | (e8[3] << 24);
                    rec.y = e8[4] | (e8[5] << 8) | (e8[6] << 16);
                    rays.push_back(rec);
                }
        int32_t fixed = -1;
        if (rooms->fixed_start && rooms->fixed_start[3 * r] >= 0) {
            const int sx = rooms->fixed_start[3 * r], sy = rooms->fixed_start[3 * r + 1],
                      sz = rooms->fixed_start[3 * r + 2];
            if (sx >= W || sy < 0 || sy >= D || sz < 0 || sz >= H)
                return fail(VN_ERR_ROOM, "room %d: start position (%d,%d,%d) outside the room", r, sx, sy, sz);
            fixed = sx | (sy << 8) | (sz << 16);
        }
        uint32_t *d = &desc[(size_t)r * 8];
        d[0] = (uint32_t)W | ((uint32_t)D << 8) | ((uint32_t)H << 16);
        d[1] = tf;
        d[2] = ray_off;
        d[3] = start_off;
        d[4] = (uint32_t)fixed;
        d[5] = (uint32_t)((W + 3) / 4) | ((uint32_t)((D + 3) / 4) << 16);
        maxW = W > maxW ? W : maxW;
        maxD = D > maxD ? D : maxD;
        maxH = H > maxH ? H : maxH;
        woff += (size_t)W * D * H;
    }

    VnEnv *e = new (std::nothrow) VnEnv();
    if (!e) return fail(VN_ERR_OOM, "host allocation failed");
    e->device = device;
    e->N = n_agents;
    e->cfg = *cfg;
    if (e->cfg.finish_percentage == 0.0) e->cfg.finish_percentage = 0.84;
    if (e->cfg.seed_stride == 0) e->cfg.seed_stride = n_agents;
    e->n_rooms = nr;
    e->total_free = total_free;
    e->nbx = (maxW + 3) / 4;
    e->nby = (maxD + 3) / 4;
    e->pw = e->nbx * 4;
    e->pd = e->nby * 4;
    e->ph = (maxH + 3) & ~3;
    e->map_bytes = (uint32_t)(e->nbx * e->nby * 16 * e->ph);

    DeviceGuard dg(device);
    int rc = ensure_mt_table(device);
    if (rc) {
        delete e;
        return rc;
    }
    // f32 obs table: (v + 2) / 22 for v = -2..20, IEEE f32 division on the host
    float lut[32];
    for (int k = 0; k < 32; ++k) {
        volatile float num = (float)(k < 23 ? k : 22);
        lut[k] = num / 22.0f;
    }
    const size_t belief_bytes = (size_t)e->map_bytes * (size_t)n_agents;
#define VN_ALLOC(ptr, bytes)                                                                    \
    do {                                                                                        \
        hipError_t e_ = hipMalloc((void **)&(ptr), (bytes));                                    \
        if (e_ != hipSuccess) {                                                                 \
            free_env(e);                                                                        \
            return fail(VN_ERR_OOM, "hipMalloc(%zu) failed: %s", (size_t)(bytes), hipGetErrorString(e_)); \
        }                                                                                       \
        e->device_bytes += (bytes);                                                             \
    } while (0)
    VN_ALLOC(e->d_rooms, desc.size() * sizeof(uint32_t));
    VN_ALLOC(e->d_rays, rays.size() * sizeof(uint2));
    VN_ALLOC(e->d_starts, starts.size() * sizeof(uint32_t));
    VN_ALLOC(e->d_lut, sizeof(lut));
    VN_ALLOC(e->d_hot, (size_t)n_agents * sizeof(uint4));
    VN_ALLOC(e->d_seed, (size_t)n_agents * sizeof(uint32_t));
    VN_ALLOC(e->d_belief, belief_bytes);
    VN_ALLOC(e->d_err, sizeof(int32_t));
#undef VN_ALLOC
    hipError_t he = hipSuccess;
    if (he == hipSuccess) he = hipMemcpy(e->d_rooms, desc.data(), desc.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemcpy(e->d_rays, rays.data(), rays.size() * sizeof(uint2), hipMemcpyHostToDevice);
    if (he == hipSuccess)
        he = hipMemcpy(e->d_starts, starts.data(), starts.size() * sizeof(uint32_t), hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemcpy(e->d_lut, lut, sizeof(lut), hipMemcpyHostToDevice);
    if (he == hipSuccess) he = hipMemset(e->d_hot, 0, (size_t)n_agents * sizeof(uint4));
    if (he == hipSuccess) he = hipMemset(e->d_seed, 0, (size_t)n_agents * sizeof(uint32_t));
    if (he == hipSuccess) he = hipMemset(e->d_belief, 0xff, belief_bytes);
    if (he == hipSuccess) he = hipMemset(e->d_err, 0, sizeof(int32_t));
    if (he == hipSuccess) he = hipDeviceSynchronize();
    if (he != hipSuccess) {
        free_env(e);
        return fail(VN_ERR_HIP, "vn_create upload: %s", hipGetErrorString(he));
    }
    *out = e;
    return VN_OK;
}

int vn_destroy(VnEnv *env) {
    if (!env) return VN_OK;
    DeviceGuard dg(env->device);
    (void)hipDeviceSynchronize();
    free_env(env);
    return VN_OK;
}

int vn_get_info(const VnEnv *env, VnInfo *info) {
    if (!env || !info) return fail(VN_ERR_INVALID, "NULL argument");
    info->n_agents = env->N;
    info->n_rooms = env->n_rooms;
    info->local_map_length = env->cfg.local_map_length;
    info->pad_w = env->pw;
    info->pad_d = env->pd;
    info->pad_h = env->ph;
    info->belief_bytes_per_agent = env->map_bytes;
    info->device_bytes = (int64_t)env->device_bytes;
    return VN_OK;
}

int vn_reset(VnEnv *env, const int64_t *seeds, const uint8_t *mask, float *obs, void *stream) {
    if (!env || !seeds || !obs) return fail(VN_ERR_INVALID, "NULL argument");
    DeviceGuard dg(env->device);
    Params p = base_params(env);
    p.seeds = seeds;
    p.mask = mask;
    p.obs = obs;
    return launch_env<true>(env, p, (hipStream_t)stream);
}

int vn_step(VnEnv *env, const int32_t *actions, float *obs, float *reward, double *reward64, uint8_t *terminated,
            uint8_t *truncated, float *terminal_obs, void *stream) {
    if (!env || !actions || !obs) return fail(VN_ERR_INVALID, "NULL argument");
    DeviceGuard dg(env->device);
    Params p = base_params(env);
    p.K = 1;
    p.actions = actions;
    p.obs = obs;
    p.reward = reward;
    p.reward64 = reward64;
    p.term = terminated;
    p.trunc = truncated;
    p.terminal_obs = terminal_obs;
    return launch_env<false>(env, p, (hipStream_t)stream);
}

int vn_step_random(VnEnv *env, uint64_t policy_seed, uint64_t t0, int32_t k_steps, int32_t *actions_out, float *obs,
                   float *reward, double *reward64, uint8_t *terminated, uint8_t *truncated, float *terminal_obs,
                   void *stream) {
    if (!env || !obs) return fail(VN_ERR_INVALID, "NULL argument");
    if (k_steps < 1) return fail(VN_ERR_INVALID, "k_steps must be >= 1 (got %d)", k_steps);
    DeviceGuard dg(env->device);
    Params p = base_params(env);
    p.K = k_steps;
    p.actions = nullptr;
    p.policy_seed = policy_seed;
    p.t0 = t0;
    p.actions_out = actions_out;
    p.obs = obs;
    p.reward = reward;
    p.reward64 = reward64;
    p.term = terminated;
    p.trunc = truncated;
    p.terminal_obs = terminal_obs;
    return launch_env<false>(env, p, (hipStream_t)stream);
}

int vn_export_state(VnEnv *env, int64_t *state_out, void *stream) {
    if (!env || !state_out) return fail(VN_ERR_INVALID, "NULL argument");
    DeviceGuard dg(env->device);
    Params p = base_params(env);
    hipLaunchKernelGGL(export_state_kernel, dim3((unsigned)((env->N + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, p, state_out);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_export_belief(VnEnv *env, int8_t *belief_out, void *stream) {
    if (!env || !belief_out) return fail(VN_ERR_INVALID, "NULL argument");
    DeviceGuard dg(env->device);
    Params p = base_params(env);
    const size_t total = (size_t)env->N * env->pw * env->pd * env->ph;
    hipLaunchKernelGGL(export_belief_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, p, belief_out, env->pw, env->pd);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int vn_gae(const float *rewards, const float *values, const float *episode_starts, const float *last_values,
           const float *dones, int32_t T, int32_t N, double gamma, double gae_lambda, float *advantages,
           float *returns, void *stream) {
    if (!rewards || !values || !episode_starts || !last_values || !dones || !advantages || !returns)
        return fail(VN_ERR_INVALID, "NULL argument");
    if (T < 1 || N < 1) return fail(VN_ERR_INVALID, "T and N must be >= 1 (got %d, %d)", T, N);
    const float g32 = (float)gamma;
    const float gl32 = (float)(gamma * gae_lambda);
    hipLaunchKernelGGL(gae_kernel, dim3((unsigned)((N + 255) / 256)), dim3(256), 0, (hipStream_t)stream, rewards,
                       values, episode_starts, last_values, dones, T, N, g32, gl32, advantages, returns);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // extern "C"
