// env_core.h -- device code shared by the CubicEnv (voxnav_env.hip) and
// simpleEnv (voxnav_simple.hip) translation units: the packed agent / room
// records, the launch parameters, CPython's MT19937 seeding restated for the
// device, the Philox policy and the obs-store helpers.  Everything is in an
// anonymous namespace: each translation unit gets its own copy (including
// the __constant__ MT table, which each unit fills through its own
// ensure_mt_table).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <new>
#include <string>
#include <type_traits>
#include <vector>

#include "vn_common.h"

// Diagnostics only: VN_ABLATE bits skip parts of the step (results invalid)
// in a separately built library (scripts/ab.py); 0 in the product.  A
// compile-time constant, so the product kernels carry no branch for it.
#ifndef VN_ABLATE
#define VN_ABLATE 0u
#endif

namespace {

using vn_detail::fail;
using vn_detail::g_last_error;

constexpr int MT_N = 624;
constexpr int MT_C = 8;  // MT words captured by the streaming seed (draws 0..7)

// init_genrand(19650218): the seed-independent prefix of CPython's
// init_by_array (Modules/_randommodule.c); filled once per device.
alignas(16) __constant__ uint32_t c_mt_g[MT_N + 8];   // + one zero block (read-ahead)

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
    uint32_t finish_visits;// smallest visited count with visited/total >= finish (f64)
    int32_t fixed_goal;    // packed "Goal" (simpleEnv) or -1
};

struct Room {
    int W, D, H;
    uint32_t total_free, ray_off, start_off, finish_visits;
    int32_t fixed_start;
    int32_t fixed_goal;
    int nbx, nby;
};

struct Agent {
    int x, y, z, facing, last_action;
    bool done, last_bump, near_wall, was_near_wall;
    uint32_t step_count, visited, bumps, move_mask;
    int cid, room;
};

// Env-constant values the (rare, out-of-line) reset path reads from device
// memory, so they need not stay live in SGPRs across the step loop.
struct EnvConst {
    const uint4 *rooms;
    const uint2 *rays;
    const uint32_t *starts;
    int32_t *err;
    int n_rooms, use_room_draw, nby, pcache;
    uint32_t agent_bytes, xp_off, map_bytes, plane_bytes;   // plane_bytes: the planes a reset clears
    const uint4 *wimg;       // plane-set mode: per room, the bricked map with latent wall bits
};

struct Params {
    const EnvConst *envc;
    uint4 *hot;
    uint32_t *next_seed;
    int8_t *belief;
    const uint4 *rooms;
    const uint2 *rays;
    const uint32_t *starts;
    const float *lut;
    int32_t *err;
    int N, L, nby, ph;
    uint32_t map_bytes;      // byte map (bricked) per agent
    uint32_t agent_bytes;    // stride: byte map + x-plane + y-plane
    uint32_t xp_off, yp_off; // plane offsets inside the agent block
    int nwx, nwy;            // u64 words per plane row
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
    uint32_t ablate;         // unused (ablations are the compile-time VN_ABLATE)
    int prio;                // step kernel: issue priority (bits, VOXNAV_ENV_PRIO; default 67)
    int dflush;              // step kernel: a step's obs flush after the next step's load issue (VOXNAV_ENV_DFLUSH)
    // simpleEnv variant
    int variant, obs_dim, pd;
    uint32_t *goal;          // per agent gx | gy<<8 | gz<<16
    uint4 *predraw;          // simpleEnv: per agent a reset draw computed ahead {start|room<<24, goal, seed, valid}
    int sbits;               // simpleEnv bit-plane layout (rooms up to 64 x 64 x 31)
    uint32_t sy_off, sz_off, qz_off;
    int sline;               // simpleEnv line layout (rooms up to 32 x 32 x 8; simple_line_kernel)
    const int8_t *wimg;      // plane-set mode (CubicEnv, PH 8, rooms <= 64 x 64): latent-wall room images
    int pcache;
    float *scratch;          // 4 KiB: targets of inactive lanes' output stores
    uint32_t *stood;         // plane-set mode PCM 2: per agent 32 words, stood-column rows (bit x of row y)
    uint2 *pnz;              // ... and per agent the plane sets whose HBM copy may be nonzero (x: rows y', y: cols x')
    int wrec_k;              // step launches of at most wrec_k steps write the window record (VOXNAV_ENV_WREC);
                             // the records follow the hot state in its allocation (wrec_base)
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
    R.finish_visits = b.z;
    R.fixed_goal = (int32_t)b.w;
    return R;
}


// Consume values in registers (an empty asm that reads them): the compiler
// then waits for their loads HERE, inside a conditional block, rather than
// carrying them as "maybe pending" into a loop, where it would wait vmcnt(0)
// -- for every load AND store in flight -- at their first use each iteration.
__device__ __forceinline__ void vn_touch(uint32_t a) { asm volatile("" ::"v"(a)); }
__device__ __forceinline__ void vn_touch(uint64_t a) { asm volatile("" ::"v"(a)); }

// every field of a room descriptor (load_room)
__device__ __forceinline__ void room_touch(const Room &R) {
    vn_touch((uint32_t)(R.W | (R.D << 8) | (R.H << 16)));
    vn_touch(R.total_free);
    vn_touch(R.ray_off);
    vn_touch(R.start_off);
    vn_touch(R.finish_visits);
    vn_touch((uint32_t)R.fixed_start);
    vn_touch((uint32_t)R.fixed_goal);
    vn_touch((uint32_t)(R.nbx | (R.nby << 16)));
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

// The two init_by_array loops are serial chains of 622 steps each (loop 2
// recomputes the loop-1 words it reads on the fly, a second chain in
// parallel).  The table words are read 8 at a time one block ahead (scalar
// loads, uniform index), so a step costs the chain's ALU latency only.
constexpr int MT_BLK = 8;

// loop 1, i = 2..623: returns p = mt[623] after loop 1
__device__ __forceinline__ uint32_t mt_loop1(uint32_t p, uint32_t seed) {
#pragma unroll
    for (int i = 2; i < MT_BLK; ++i) p = mix1(c_mt_g[i], p, seed);
    const uint4 *G = reinterpret_cast<const uint4 *>(c_mt_g);
    uint4 c0 = G[MT_BLK / 4], c1 = G[MT_BLK / 4 + 1];
    for (int i = MT_BLK; i < MT_N; i += MT_BLK) {
        const uint4 n0 = G[(i + MT_BLK) / 4], n1 = G[(i + MT_BLK) / 4 + 1];   // table padded by one block
        p = mix1(c0.x, p, seed);
        p = mix1(c0.y, p, seed);
        p = mix1(c0.z, p, seed);
        p = mix1(c0.w, p, seed);
        p = mix1(c1.x, p, seed);
        p = mix1(c1.y, p, seed);
        p = mix1(c1.z, p, seed);
        p = mix1(c1.w, p, seed);
        c0 = n0;
        c1 = n1;
    }
    return p;
}

// loop 2 over i in [a, b) without captures (p1: loop-1 word chain, q: new words)
__device__ __forceinline__ void mt_loop2(uint32_t &p1, uint32_t &q, int a, int b, uint32_t seed) {
    int i = a;
    for (; i < b && (i & (MT_BLK - 1)); ++i) {
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
    }
    const uint4 *G = reinterpret_cast<const uint4 *>(c_mt_g);
    if (i + MT_BLK <= b) {
        uint4 c0 = G[i / 4], c1 = G[i / 4 + 1];
        for (; i + MT_BLK <= b; i += MT_BLK) {
            const uint4 n0 = G[(i + MT_BLK) / 4], n1 = G[(i + MT_BLK) / 4 + 1];
            const uint32_t gw[MT_BLK] = {c0.x, c0.y, c0.z, c0.w, c1.x, c1.y, c1.z, c1.w};
#pragma unroll
            for (int k = 0; k < MT_BLK; ++k) {
                p1 = mix1(gw[k], p1, seed);
                q = mix2(p1, q, (uint32_t)(i + k));
            }
            c0 = n0;
            c1 = n1;
        }
    }
    for (; i < b; ++i) {
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
    }
}

// Outputs [j0, j0 + MT_C) of the first twist of random.seed(seed);
// j0 % MT_C == 0 and j0 + MT_C <= 227 (the first twist's outputs that read
// only final state words).  One pass over the two loops.
struct MtBlock {            // returned by value: stays in VGPRs across the call
    uint32_t w[MT_C];
};

__device__ __forceinline__ MtBlock mt_outputs_inl(uint32_t seed, int j0);
__device__ MtBlock mt_outputs(uint32_t seed, int j0) { return mt_outputs_inl(seed, j0); }
__device__ __forceinline__ MtBlock mt_outputs_inl(uint32_t seed, int j0) {
    MtBlock out;
    uint32_t p = mix1(c_mt_g[1], c_mt_g[0], seed);
    const uint32_t m1_1 = p;
    p = mt_loop1(p, seed);
    const uint32_t m1b1 = mix1(m1_1, p, seed);  // wrap: i = 1 again, mt[0] = mt[623]
    uint32_t p1 = m1_1, q = m1b1;
    uint32_t lo[MT_C + 1], hi[MT_C];            // F[j0 .. j0+MT_C], F[j0+397 .. j0+397+MT_C-1]
    if (j0 == 0) {
#pragma unroll
        for (int i = 2; i <= MT_C; ++i) {
            p1 = mix1(c_mt_g[i], p1, seed);
            q = mix2(p1, q, (uint32_t)i);
            lo[i] = q;
        }
    } else {
        mt_loop2(p1, q, 2, j0, seed);
#pragma unroll
        for (int k = 0; k <= MT_C; ++k) {
            p1 = mix1(c_mt_g[j0 + k], p1, seed);
            q = mix2(p1, q, (uint32_t)(j0 + k));
            lo[k] = q;
        }
    }
    mt_loop2(p1, q, j0 + MT_C + 1, 397 + j0, seed);
#pragma unroll
    for (int k = 0; k < MT_C; ++k) {
        const int i = 397 + j0 + k;
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
        hi[k] = q;
    }
    mt_loop2(p1, q, 397 + j0 + MT_C, MT_N, seed);
    if (j0 == 0) {
        lo[1] = mix2(m1b1, q, 1u);              // F[1]: loop 2's wrap step
        lo[0] = 0x80000000u;                    // F[0]
    }
#pragma unroll
    for (int j = 0; j < MT_C; ++j) {
        const uint32_t y = (lo[j] & 0x80000000u) | (lo[j + 1] & 0x7fffffffu);
        out.w[j] = mt_temper(hi[j] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
    }
    return out;
}

__device__ __forceinline__ void mt_first_outputs(uint32_t seed, uint32_t out[MT_C]) {
    const MtBlock b = mt_outputs(seed, 0);
#pragma unroll
    for (int j = 0; j < MT_C; ++j) out[j] = b.w[j];
}

// the next block of outputs, one pass (rejection sampling ran past the buffer)
__device__ __noinline__ MtBlock mt_refill(uint32_t seed, int j0, int32_t *err) {
    if (j0 + MT_C > MT_N - 397) {
        atomicOr(err, 1);
        MtBlock z;
#pragma unroll
        for (int j = 0; j < MT_C; ++j) z.w[j] = 0u;
        return z;
    }
    return mt_outputs(seed, j0);
}

// INL: the refill inlined (no call: a kernel whose step loop must not spill
// around a call site)
template <bool INL = false>
struct MtStreamT {
    uint32_t seed;
    uint32_t buf[MT_C];
    int used;
    int32_t *err;

    __device__ uint32_t next() {
        if (used > 0 && (used % MT_C) == 0) {
            MtBlock b;
            if constexpr (INL) {
                if (used + MT_C > MT_N - 397) {
                    atomicOr(err, 1);
#pragma unroll
                    for (int j = 0; j < MT_C; ++j) b.w[j] = 0u;
                } else {
                    b = mt_outputs_inl(seed, used);
                }
            } else {
                b = mt_refill(seed, used, err);
            }
#pragma unroll
            for (int j = 0; j < MT_C; ++j) buf[j] = b.w[j];
        }
        const uint32_t r = buf[0];
#pragma unroll
        for (int t = 0; t < MT_C - 1; ++t) buf[t] = buf[t + 1];
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
using MtStream = MtStreamT<false>;

// ----------------------------------------------------------------------------
// Philox4x32-10 random policy (build-defined): one call per
// agent per 4 steps, counter = (global agent id, t / 4), word t % 4,
// action = (word * 6) >> 32.
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint4 philox4x32_10(uint64_t key, uint64_t gid, uint64_t blk) {
    uint32_t c0 = (uint32_t)gid, c1 = (uint32_t)(gid >> 32), c2 = (uint32_t)blk, c3 = (uint32_t)(blk >> 32);
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
    return make_uint4(c0, c1, c2, c3);
}

// ----------------------------------------------------------------------------
// Agent groups: 4 lanes per agent (16 agents per wave64).
//
// Lane q of an agent owns window row dy = q - 2: it loads the 4 columns
// (x+i-2, y+q-2), i = 0..3 (z contiguous, one 8/16/32-byte access each) and
// writes obs[16i+4q .. 16i+4q+3] -- the 4 lanes of an agent store 64
// contiguous bytes per instruction.  The horizontal ray cells beyond the
// window are spread over the 4 lanes (4 consecutive cells of one ray per
// instruction), so every wave instruction touches ~1-2 cache lines per agent.
// Control state (pose, counters, flags, reward) is held redundantly by the
// 4 lanes.
//
// Belief byte encoding (OR-able):  bit7 = known, bit6 = wall, bits0-5 =
// visit count (saturating at 63; obs clips at 20, reward caps at 25).
//   unknown (-1) = 0x00, known free (0) = 0x80, visited n = 0x80|n,
//   known wall (-2) = 0xC0.
// Sensing marks a free cell by OR 0x80 and the first wall by OR 0xC0,
// idempotent, so a cell already known is never rewritten.
// ----------------------------------------------------------------------------
constexpr int GROUP = 4;
constexpr uint32_t KNOWN = 0x80u, WALLB = 0xC0u;
// LDS table: [0,256) obs value of each belief byte; [256,262) f32(a/5);
// [264,281) f32(c/L)   (get_obs :273-275, :284, :287)
constexpr int TAB_ACTION = 256, TAB_CID = 264, TAB_SIZE = 288;
// after the CubicEnv table in the same device buffer: the simpleEnv reward of
// each event code (bit 0 bump, 1 repeated move, 2 goal, 3 explored), 16 f32
// then 16 f64, each the reference's f64 sum in its order (envs/simpleEnv.py:189-217)
constexpr int TAB_SREW = TAB_SIZE, TAB_SREW64 = TAB_SIZE + 16, TAB_ALL = TAB_SIZE + 48;

__device__ __forceinline__ int decode_count(uint32_t b) {   // center cell: known free or unknown
    return (b & KNOWN) ? (int)(b & 0x3fu) : -1;
}

typedef float F4v __attribute__((ext_vector_type(4)));

// LDS position of LUT entry b: the common belief bytes 0x00 / 0x40 / 0x80 /
// 0xC0 (unknown, latent wall, free, wall) would all sit in LDS bank 0 and a
// 32-lane lookup would serialise over them; XOR-ing the low 2 bits with the
// top 2 puts them in banks 0-3 (a permutation inside every aligned 4-group).
#ifndef VN_TAB_SWZ
#define VN_TAB_SWZ 1
#endif
__device__ __forceinline__ uint32_t tab_ix(uint32_t b) { return VN_TAB_SWZ ? b ^ ((b >> 6) & 3u) : b; }

// float4 of a code word (4 belief bytes or tail codes): 4 LUT lookups
__device__ __forceinline__ float4 code_float4(uint32_t wb, const float *tab) {
    if (VN_TAB_SWZ) wb ^= (wb >> 6) & 0x03030303u;        // tab_ix of all 4 bytes
    return make_float4(tab[wb & 0xffu], tab[(wb >> 8) & 0xffu], tab[(wb >> 16) & 0xffu], tab[wb >> 24]);
}

// Streaming store of one obs float4 to HBM.  VN_OBS_STORE: 0 plain, 1
// non-temporal, 2 sc1 (write-through; the line is dropped from L2, so the
// obs stream does not evict the belief / plane / ray-table lines), 3 sc1 nt,
// 4 sc0 sc1 nt.  Measured (scripts/ab.py, 65536 agents, 32x32x8, 5408
// steps, 7 rounds): 1 = 6.83, 3 = 6.86, 4 = 6.65 G env-steps/s -- equal
// within noise; 0 and 2 are ~15% slower.  1 stays the default.
#ifndef VN_OBS_STORE
#define VN_OBS_STORE 1
#endif
__device__ __forceinline__ void obs_store(float4 *dst, const float4 &v) {
#if VN_OBS_STORE == 1
    __builtin_nontemporal_store(F4v{v.x, v.y, v.z, v.w}, reinterpret_cast<F4v *>(dst));
#elif VN_OBS_STORE == 2
    const F4v w{v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(dst), "v"(w) : "memory");
#elif VN_OBS_STORE == 3
    const F4v w{v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc1 nt" ::"v"(dst), "v"(w) : "memory");
#elif VN_OBS_STORE == 4
    const F4v w{v.x, v.y, v.z, v.w};
    asm volatile("global_store_dwordx4 %0, %1, off sc0 sc1 nt" ::"v"(dst), "v"(w) : "memory");
#else
    *dst = v;
#endif
}
typedef __attribute__((address_space(3))) F4v LdsF4;     // LDS
typedef __attribute__((address_space(1))) F4v GlbF4;     // global
typedef __attribute__((address_space(3))) uint32_t LdsU32;  // LDS
__device__ __forceinline__ F4v f4v(const float4 &v) { return F4v{v.x, v.y, v.z, v.w}; }

__device__ __forceinline__ Room load_room_c(const EnvConst *ec, int r) {
    const uint4 a = ec->rooms[2 * r];
    const uint4 b = ec->rooms[2 * r + 1];
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
    R.finish_visits = b.z;
    R.fixed_goal = (int32_t)b.w;
    return R;
}

// host: this translation unit's copy of the MT table (c_mt_g), once per device
bool g_mt_ready[64] = {false};

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

}  // namespace

// the simpleEnv unit (voxnav_simple.hip), called by voxnav_env.hip's host side
namespace vn_simple {
int ensure_mt(int device);
int launch(bool reset_only, int sline, int sbits, int L, int N, int obs_dim, const void *params, hipStream_t s);
std::string label(bool reset_only, bool ext, int sline, int sbits, int L);
int export_belief(const void *params, int8_t *out, int pw, int pd, hipStream_t s);
}  // namespace vn_simple
