// voxnav_simple.hip -- MI355X (gfx950) kernels of the simpleEnv variant
// (envs/simpleEnv.py).  Split from voxnav_env.hip:
// the CubicEnv step kernel and the C-ABI stay there; this unit holds the
// simpleEnv step kernels (line layout for rooms <= 32 x 32 x 8, word layout
// up to 64 x 64 x 31, dense maps beyond), their reset kernel and belief
// export, and the launcher voxnav_env.hip's launch_env calls.

#include "env_core.h"

namespace {

// ============================================================================
// simpleEnv variant (envs/simpleEnv.py): walls are
// the room file's `2` tokens, the belief map holds the reference's
// internal_grid values as int8 (-1 unknown, 0 free, 1 visited, 2 wall),
// dense per agent [pd-major: x][y][z] with z contiguous (PH bytes).  The
// observation is 6 rays x L belief values + 6 distances + last_action
// (obs_dim = 6L + 7).  One lane per agent, 64 agents per block; obs rows are
// staged in LDS and written as one contiguous span per block.
// ============================================================================

// absolute ray directions of the relative moves (envs/simpleEnv.py:153-158,
// :224-231) in the ray-record byte order 0:+x 1:-x 2:+y 3:-y 4:+z 5:-z
constexpr int kRelDir[4][4] = {
    {2, 0, 3, 1},   // forward  (N, E, S, W)
    {0, 3, 1, 2},   // right
    {3, 1, 2, 0},   // backward
    {1, 2, 0, 3},   // left
};
constexpr uint32_t pack_rel_dir() {
    uint32_t v = 0;
    for (int a = 0; a < 4; ++a)
        for (int f = 0; f < 4; ++f) v |= (uint32_t)kRelDir[a][f] << (2 * (4 * a + f));
    return v;
}
// 2-bit fields in one immediate: no memory lookups on the step's critical path
__device__ __forceinline__ int rel_dir(int a, int facing) {
    return (int)((pack_rel_dir() >> (2 * (4 * a + facing))) & 3u);
}
// +x -> east(1), -x -> west(3), +y -> north(0), -y -> south(2)
__device__ __forceinline__ int facing_of(int d) { return (int)((0x8Du >> (2 * d)) & 3u); }

// obs slot of absolute direction j < 4 for facing f: slot k with rel_dir of
// [fwd, left, right, back][k] == j
constexpr uint32_t pack_obs_slot() {
    uint32_t v = 0;
    const int rel_of_slot[4] = {0, 3, 1, 2};   // forward, left, right, backward (action indices)
    for (int f = 0; f < 4; ++f)
        for (int k = 0; k < 4; ++k) v |= (uint32_t)k << (2 * (4 * f + kRelDir[rel_of_slot[k]][f]));
    return v;
}
__device__ __forceinline__ int obs_slot(int j, int facing) {
    return j >= 4 ? j : (int)((pack_obs_slot() >> (2 * (4 * facing + j))) & 3u);
}


// MT draws of simpleEnv's load_room (:350, :410-426): room, start (drawn if
// absent or on a wall), goal (drawn if absent or on a wall).  Returns
// (start | room<<24, goal).
template <bool INL>
__device__ __attribute__((always_inline)) inline uint2 simple_draw_t(const EnvConst *ec, uint32_t seed);
template <typename MT>
__device__ __attribute__((always_inline)) inline uint2 simple_draw_from(const EnvConst *ec, MT &mt);
__device__ __noinline__ uint2 simple_draw(const EnvConst *ec, uint32_t seed) { return simple_draw_t<false>(ec, seed); }
template <bool INL>
__device__ __attribute__((always_inline)) inline uint2 simple_draw_t(const EnvConst *ec, uint32_t seed) {
    MtStreamT<INL> mt;
    mt.seed = seed;
    mt.used = 0;
    mt.err = ec->err;
    if constexpr (INL) {
        const MtBlock b0 = mt_outputs_inl(seed, 0);
#pragma unroll
        for (int j = 0; j < MT_C; ++j) mt.buf[j] = b0.w[j];
    } else {
        mt_first_outputs(seed, mt.buf);
    }
    return simple_draw_from(ec, mt);
}

// The first MT_W = 24 outputs of random.seed(seed) in ONE pass of the two
// init_by_array chains (mt_outputs captures 8 per pass; a wave-wide draw of
// 64 lanes would otherwise re-run the chains whenever any lane's rejection
// sampling passed 8 outputs), written to the lane's LDS row (stride MT_WS).
constexpr int MT_W = 24, MT_WS = 25;
__device__ __noinline__ void mt_outputs_wide(uint32_t seed, uint32_t *lds_row) {
    uint32_t p = mix1(c_mt_g[1], c_mt_g[0], seed);
    const uint32_t m1_1 = p;
    p = mt_loop1(p, seed);
    const uint32_t m1b1 = mix1(m1_1, p, seed);   // wrap: i = 1 again, mt[0] = mt[623]
    uint32_t p1 = m1_1, q = m1b1;
    uint32_t lo[MT_W + 1], hi[MT_W];             // F[0 .. MT_W], F[397 .. 397 + MT_W - 1]
#pragma unroll
    for (int i = 2; i <= MT_W; ++i) {
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
        lo[i] = q;
    }
    mt_loop2(p1, q, MT_W + 1, 397, seed);
#pragma unroll
    for (int k = 0; k < MT_W; ++k) {
        const int i = 397 + k;
        p1 = mix1(c_mt_g[i], p1, seed);
        q = mix2(p1, q, (uint32_t)i);
        hi[k] = q;
    }
    mt_loop2(p1, q, 397 + MT_W, MT_N, seed);
    lo[1] = mix2(m1b1, q, 1u);                   // F[1]: loop 2's wrap step
    lo[0] = 0x80000000u;                         // F[0]
#pragma unroll
    for (int j = 0; j < MT_W; ++j) {
        const uint32_t y = (lo[j] & 0x80000000u) | (lo[j + 1] & 0x7fffffffu);
        lds_row[j] = mt_temper(hi[j] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u));
    }
}

// MT output stream over a lane's LDS row of MT_W outputs (mt_outputs_wide),
// blocks past it recomputed one at a time (mt_refill)
struct MtLdsStream {
    const uint32_t *row;
    uint32_t seed;
    int used;
    int32_t *err;
    MtBlock ext;
    __device__ uint32_t next() {
        uint32_t r;
        if (used < MT_W) {
            r = row[used];
        } else {
            if ((used % MT_C) == 0) ext = mt_refill(seed, used, err);
            const int j = used % MT_C;
            r = ext.w[0];
#pragma unroll
            for (int t = 1; t < MT_C; ++t) r = j == t ? ext.w[t] : r;
        }
        ++used;
        return r;
    }
    __device__ uint32_t below(uint32_t n) {
        const int k = 32 - __clz(n);
        uint32_t r = next() >> (32 - k);
        while (r >= n) r = next() >> (32 - k);
        return r;
    }
};

template <typename MT>
__device__ __attribute__((always_inline)) inline uint2 simple_draw_from(const EnvConst *ec, MT &mt) {
    const int room = ec->use_room_draw ? (int)mt.below((uint32_t)ec->n_rooms) : 0;
    const Room R = load_room_c(ec, room);
    auto is_wall = [&](uint32_t c) {
        const int x = c & 0xff, y = (c >> 8) & 0xff, z = (c >> 16) & 0xff;
        return ((ec->rays[R.ray_off + (uint32_t)((x * R.D + y) * R.H + z)].y >> 16) & 1u) != 0u;
    };
    uint32_t s = R.fixed_start >= 0 ? (uint32_t)R.fixed_start : ec->starts[R.start_off + mt.below(R.total_free)];
    if (is_wall(s)) s = ec->starts[R.start_off + mt.below(R.total_free)];
    uint32_t gl = R.fixed_goal >= 0 ? (uint32_t)R.fixed_goal : ec->starts[R.start_off + mt.below(R.total_free)];
    if (is_wall(gl)) gl = ec->starts[R.start_off + mt.below(R.total_free)];
    return make_uint2((s & 0xffffffu) | ((uint32_t)room << 24), gl & 0xffffffu);
}

// _sense_direction (:301-337) along absolute direction d from the agent's
// cell, using the cell's ray record (free run n to the first wall / edge).
// Writes L obs values, returns the distance count * 0.25.
__device__ __forceinline__ float simple_ray(int8_t *map, const Params &p, int cell, uint2 rec, int d, float *out) {
    const uint32_t e8 = ((d < 4 ? rec.x : rec.y) >> (8 * (d & 3))) & 0xffu;
    const int n = (int)(e8 & 0x7fu);
    const bool at_wall = (e8 & 0x80u) != 0u;
    const int L = p.L;
    const int sx = p.pd * p.ph, sy = p.ph;
    const int stride = d == 0 ? sx : d == 1 ? -sx : d == 2 ? sy : d == 3 ? -sy : d == 4 ? 1 : -1;
    const int m = n < L ? n : L;
    int c = cell;
    for (int s = 0; s < m; ++s) {
        c += stride;
        int v = map[c];
        if (v == -1) {           // unknown -> known free (:328-329)
            map[c] = 0;
            v = 0;
        }
        out[s] = (float)v;
    }
    if (n < L) {
        if (at_wall) map[c + stride] = 2;   // first wall (:321-324)
        else if (n >= 1) map[c] = 2;        // edge: the last in-room cell becomes a wall (:311-319)
        out[n] = 2.0f;
        for (int s = n + 1; s < L; ++s) out[s] = -1.0f;
    }
    return (float)((double)m * 0.25);       // round(count * cell_size, 2) (:337)
}

__device__ __forceinline__ void simple_observe(int8_t *map, const Params &p, const Agent &g, const Room &R,
                                               float *row) {
    const uint2 rec = p.rays[R.ray_off + (uint32_t)((g.x * R.D + g.y) * R.H + g.z)];
    const int cell = (g.x * p.pd + g.y) * p.ph + g.z;
    const int L = p.L;
    const int dirs[6] = {rel_dir(0, g.facing), rel_dir(3, g.facing), rel_dir(1, g.facing),
                         rel_dir(2, g.facing), 4, 5};   // forward, left, right, backward, up, down (:233)
#pragma unroll
    for (int k = 0; k < 6; ++k) row[6 * L + k] = simple_ray(map, p, cell, rec, dirs[k], row + k * L);
    row[6 * L + 6] = (float)g.last_action;
}

// reset for the lanes with `need`: draws, the wave clears every resetting
// agent's map rows x < W (all 64 lanes per agent, 8-byte stores), then each
// agent marks its start cell visited and senses (reset + get_obs(), as the
// reference's callers do, train/evaluate_grid.py:54-55).
__device__ void simple_reset_wave(const Params &p, int8_t *map, bool need, uint32_t seed, Agent &g,
                                  uint32_t &goal, Room &R, float *row, int lane, int block_agent0) {
    uint2 drawn = make_uint2(0u, 0u);
    if (need) drawn = simple_draw(p.envc, seed);
    uint64_t m = __ballot(need);
    while (m) {
        const int src = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        const int room = __shfl((int)(drawn.x >> 24), src);
        const Room Rr = load_room(p, room);
        uint64_t *base = reinterpret_cast<uint64_t *>(p.belief + (size_t)(block_agent0 + src) * p.agent_bytes);
        const uint32_t words = (uint32_t)(Rr.W * p.pd * p.ph) >> 3;
        for (uint32_t w = (uint32_t)lane; w < words; w += 64u) base[w] = ~0ull;   // -1 = unknown (:85)
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (need) {
        g.room = (int)(drawn.x >> 24);
        R = load_room(p, g.room);
        g.x = drawn.x & 0xff;
        g.y = (drawn.x >> 8) & 0xff;
        g.z = (drawn.x >> 16) & 0xff;
        goal = drawn.y;
        g.facing = 0;
        g.last_action = 0;
        g.done = g.last_bump = g.near_wall = g.was_near_wall = false;
        g.step_count = 0;
        g.visited = 1;
        g.bumps = 0;
        g.cid = 0;
        g.move_mask = 0;
        map[(g.x * p.pd + g.y) * p.ph + g.z] = 1;                              // :86
        simple_observe(map, p, g, R, row);
    }
}

template <bool RESET_ONLY>
__global__ __launch_bounds__(64) void simple_kernel(Params p) {
    extern __shared__ float sstage[];   // [64][obs_dim]
    const int lane = threadIdx.x;
    const int a0 = blockIdx.x * 64;
    const int ai = a0 + lane;
    const bool live = ai < p.N;
    const int OD = p.obs_dim, L = p.L;
    const int rows = min(64, p.N - a0);
    float *row = sstage + lane * OD;
    int8_t *map = p.belief + (size_t)(live ? ai : a0) * p.agent_bytes;
    Agent g = unpack(live ? p.hot[ai] : make_uint4(0u, 0u, 0u, 0u));
    uint32_t goal = live ? p.goal[ai] : 0u;
    uint32_t next_seed = live ? p.next_seed[ai] : 0u;
    Room R = load_room(p, g.room);

    if (RESET_ONLY) {
        const bool need = live && (!p.mask || p.mask[ai]);
        const uint32_t seed = need ? (uint32_t)p.seeds[ai] : 0u;
        simple_reset_wave(p, map, need, seed, g, goal, R, row, lane, a0);
        if (need) {
            float *o = p.obs + (size_t)ai * OD;
            for (int k = 0; k < OD; ++k) o[k] = row[k];
            p.hot[ai] = pack(g);
            p.goal[ai] = goal;
            p.next_seed[ai] = seed + p.seed_stride;   // modulo 2^32
        }
        return;
    }

    for (int k = 0; k < p.K; ++k) {
        const uint64_t t = p.t0 + (uint64_t)k;
        int a = 0;
        if (live) {
            if (p.actions) {
                a = p.actions[(size_t)k * p.N + ai];
            } else {
                const uint4 w = philox4x32_10(p.policy_seed, p.gid_base + (uint64_t)ai, t >> 2);
                const uint32_t word = (t & 3) == 0 ? w.x : (t & 3) == 1 ? w.y : (t & 3) == 2 ? w.z : w.w;
                a = (int)(((uint64_t)word * 6u) >> 32);
            }
            if (p.actions_out) p.actions_out[(size_t)k * p.N + ai] = a;
        }
        bool trunc = false, term = false;
        double r = 0.0;
        if (live) {
            // step (:109-150)
            g.step_count += 1;
            trunc = g.step_count >= R.total_free;                      // :111, max_steps = total_free (:409)
            const int d = a < 4 ? rel_dir(a, g.facing) : (a == 4 ? 4 : 5);
            if (a < 4) g.facing = facing_of(d);                        // :164-171
            const uint2 rec = p.rays[R.ray_off + (uint32_t)((g.x * R.D + g.y) * R.H + g.z)];
            const uint32_t e8 = ((d < 4 ? rec.x : rec.y) >> (8 * (d & 3))) & 0x7fu;
            bool bumped = false, explored = false;
            if (e8 >= 1u) {                                              // _mark_visited (:273-298)
                g.x += d == 0 ? 1 : d == 1 ? -1 : 0;
                g.y += d == 2 ? 1 : d == 3 ? -1 : 0;
                g.z += d == 4 ? 1 : d == 5 ? -1 : 0;
                int8_t *c = map + (g.x * p.pd + g.y) * p.ph + g.z;
                const int v = *c;
                if (v == 0 || v == -1) {
                    *c = 1;
                    g.visited += 1;
                    explored = true;
                }
            } else {
                bumped = true;
            }
            g.last_action = a;                                           // :137
            simple_observe(map, p, g, R, row);                           // :139
            // compute_reward (:189-217), f64 in the reference's order
            r = -0.1;
            if (bumped) {
                g.bumps += 1;
                r += -10.0;
            }
            if (a != 2 && a < 4) r += 0.05;                              // last_action == a here
            const int gx = goal & 0xff, gy = (goal >> 8) & 0xff, gz = (goal >> 16) & 0xff;
            if (g.x == gx && g.y == gy && g.z >= gz && g.z - gz < 5) {   // SPOT_GOAL_HEIGTH = 5 (:201-206)
                g.done = true;
                r += 100.0;
            }
            if (trunc) r += 0.0;                                         // r += -0
            if (explored) r += 1.0;
            term = g.done;
            const size_t o = (size_t)k * p.N + ai;
            if (p.reward) p.reward[o] = (float)r;
            if (p.reward64) p.reward64[o] = r;
            if (p.term) p.term[o] = term;
            if (p.trunc) p.trunc[o] = trunc;
            if ((term || trunc) && p.autoreset && p.terminal_obs) {
                float *to = p.terminal_obs + o * OD;
                for (int q = 0; q < OD; ++q) to[q] = row[q];
            }
        }
        // SB3 VecEnv auto-reset
        const bool need = live && p.autoreset && (term || trunc);
        if (__ballot(need)) {
            simple_reset_wave(p, map, need, next_seed, g, goal, R, row, lane, a0);
            if (need) next_seed += p.seed_stride;
        }
        __syncthreads();
        float *dst = p.obs + ((size_t)k * p.N + a0) * OD;
        for (int q = lane; q < rows * OD; q += 64) dst[q] = sstage[q];
        __syncthreads();
    }
    if (live) {
        p.hot[ai] = pack(g);
        p.goal[ai] = goal;
        p.next_seed[ai] = next_seed;
    }
    (void)L;
}

// ============================================================================
// simpleEnv, bit-plane layout (rooms up to 64 x 64 x 31; larger rooms use the
// dense kernel above).  The belief map is not stored as bytes.  Per agent:
//   S  the agent has stood on the cell: internal_grid == 1 (:86, :294), or a
//      visited cell the edge quirk later turned into 2.  Kept in three axis
//      planes so that a ray along any axis is one word:
//      SX[y][z] (bit x, u64), SY[x][z] (bit y, u64), SZ[x][y] (bit z, u32)
//   Q  edge-quirk mark: the last in-room cell of a ray that leaves the room
//      becomes 2 (:311-319).  QZ[x][y] (bit z, u32); agent flag in hot.w
// Every other internal_grid value is a function of S, Q and the walls: the
// positions the agent has sensed from are exactly its S cells (reset and
// every step observe where the agent stands, and every such cell is marked),
// so a cell is known -- 0 if free, 2 if wall -- iff an S cell lies within L
// cells of it along an axis with only free cells in between (:301-337).
// export_belief derives the map; the step reads only S and Q.  In-run obs
// values: Q ? 2 : S ? 1 : 0.
// ============================================================================
struct SPlanes {
    uint64_t *sx, *sy;
    uint32_t *sz, *qz;
};

__device__ __forceinline__ SPlanes splanes(const Params &p, int agent) {
    int8_t *b = p.belief + (size_t)agent * p.agent_bytes;
    SPlanes q;
    q.sx = reinterpret_cast<uint64_t *>(b);
    q.sy = reinterpret_cast<uint64_t *>(b + p.sy_off);
    q.sz = reinterpret_cast<uint32_t *>(b + p.sz_off);
    q.qz = reinterpret_cast<uint32_t *>(b + p.qz_off);
    return q;
}

// cached S words through the agent's cell + the cell's ray record
struct SRows {
    uint64_t wx, wy;
    uint32_t wz;
    uint2 rec;
};

__device__ __forceinline__ uint32_t ray_e8(uint2 rec, int d) {
    return ((d < 4 ? rec.x : rec.y) >> (8 * (d & 3))) & 0xffu;
}

// simple_ray on the bit planes: obs values of ray d (L floats) from the S
// word along the ray axis, Q bits looked up only when the agent has any;
// then the edge-quirk mark.  Returns count * 0.25.
// (scalars by value: a select over struct fields folds into a dynamic load
// from a stack copy of the struct)
template <int LMAX>
__device__ __forceinline__ float sb_ray(const Params &p, const SPlanes &pl, int gx, int gy, int gz, bool hasq,
                                        uint64_t wx, uint64_t wy, uint32_t wz, uint2 rec, int d, float *out,
                                        bool &newq) {
    const uint32_t e8 = ray_e8(rec, d);
    const int n = (int)(e8 & 0x7fu);
    const int L = p.L;
    const int m = n < L ? n : L;
    const int ax = d >> 1;
    const int sgn = (d & 1) ? -1 : 1;
    const uint64_t run = ax == 0 ? wx : ax == 1 ? wy : (uint64_t)wz;
    const int pos = ax == 0 ? gx : ax == 1 ? gy : gz;
#pragma unroll
    for (int s = 0; s < LMAX; ++s) {
        if (s >= L) break;
        float v;
        if (s < m) {
            const int c = pos + sgn * (s + 1);
            uint32_t b = (uint32_t)(run >> c) & 1u;
            if (hasq) {
                const int qx = ax == 0 ? c : gx, qy = ax == 1 ? c : gy, qzz = ax == 2 ? c : gz;
                if ((pl.qz[qx * p.pd + qy] >> qzz) & 1u) b = 2u;
            }
            v = (float)b;
        } else {
            v = s == n ? 2.0f : -1.0f;   // wall / edge terminator, then padding (:321-331)
        }
        out[s] = v;
    }
    if (n < L && !(e8 & 0x80u) && n >= 1) {   // edge quirk (:311-319)
        const int c = pos + sgn * n;
        const int qx = ax == 0 ? c : gx, qy = ax == 1 ? c : gy, qzz = ax == 2 ? c : gz;
        uint32_t *q = pl.qz + qx * p.pd + qy;
        // no Q bit anywhere yet -> the word is 0 (up and down share a column)
        const uint32_t old = (hasq || newq) ? *q : 0u;
        if (!((old >> qzz) & 1u)) *q = old | (1u << qzz);
        newq = true;
    }
    return (float)m * 0.25f;                 // round(count * 0.25, 2) is exact
}

template <int LMAX>
__device__ __forceinline__ void sb_observe(const Params &p, const SPlanes &pl, Agent &g, const SRows &w, float *row) {
    const int L = p.L;
    const bool hasq = g.move_mask & 1u;
    bool newq = false;
    const int dirs[6] = {rel_dir(0, g.facing), rel_dir(3, g.facing), rel_dir(1, g.facing),
                         rel_dir(2, g.facing), 4, 5};   // forward, left, right, backward, up, down (:233)
#pragma unroll
    for (int k = 0; k < 6; ++k)
        row[6 * L + k] = sb_ray<LMAX>(p, pl, g.x, g.y, g.z, hasq, w.wx, w.wy, w.wz, w.rec, dirs[k], row + k * L, newq);
    row[6 * L + 6] = (float)g.last_action;
    if (newq) g.move_mask |= 1u;
}

// sb_observe without divergent branches, for waves in which no lane has Q
// marks or stands where a ray ends at the room's edge (ray record bit 17):
// the rays in ABSOLUTE directions (ray axis, sign and S word fixed per ray),
// each written at the obs slot the agent's facing gives it (obs_slot).  Per
// ray cell s < L: the S bit if s < min(n, L), else 2 at s == n (wall), else -1
// (:301-337).  Otherwise the wave takes sb_observe.
template <int LMAX>
__device__ __forceinline__ void sp_observe(const Params &p, const SPlanes &pl, Agent &g, const SRows &w, float *row) {
    const bool slow = (g.move_mask & 1u) || ((w.rec.y >> 17) & 1u);
    if (__builtin_expect(__ballot(slow) != 0ull, 0)) {
        sb_observe<LMAX>(p, pl, g, w, row);
        return;
    }
    const int L = p.L;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t e8 = ray_e8(w.rec, j);
        const int n = (int)(e8 & 0x7fu);
        const int m = n < L ? n : L;
        // t: bit s = the S bit of ray cell s + 1
        uint32_t t;
        if (j == 0) t = (uint32_t)(w.wx >> ((g.x + 1) & 63));
        else if (j == 2) t = (uint32_t)(w.wy >> ((g.y + 1) & 63));
        else if (j == 4) t = w.wz >> ((g.z + 1) & 31);
        else if (j == 1) t = __builtin_bitreverse32((uint32_t)((w.wx << ((64 - g.x) & 63)) >> 32));
        else if (j == 3) t = __builtin_bitreverse32((uint32_t)((w.wy << ((64 - g.y) & 63)) >> 32));
        else t = __builtin_bitreverse32(w.wz << ((32 - g.z) & 31));
        float *out = row + obs_slot(j, g.facing) * L;
#pragma unroll
        for (int s = 0; s < LMAX; ++s) {
            if (s >= L) break;
            const float fb = ((t >> s) & 1u) ? 1.0f : 0.0f;
            const float pad = s == n ? 2.0f : -1.0f;
            out[s] = s < m ? fb : pad;
        }
        row[6 * L + obs_slot(j, g.facing)] = (float)m * 0.25f;   // round(count * 0.25, 2) is exact
    }
    row[6 * L + 6] = (float)g.last_action;
}

// Four ray cells at once: entry (bits | (clamp(m - 4c, -1, 4) + 1) << 4) of
// the table holds the obs values of cells 4c..4c+3 of a ray with min(n, L) = m
// free cells whose S bits (cells 4c..4c+3) are `bits`: the S bit below m, 2 at
// m (the wall / edge terminator -- only reached when n < L), -1 beyond.
constexpr int SL_CLUT = 96;
__device__ __forceinline__ void sl_build_cell_lut(float4 *lut, int lane) {
    for (int e = lane; e < SL_CLUT; e += 64) {
        const int bits = e & 15, r = (e >> 4) - 1;
        float v[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = i < r ? (float)((bits >> i) & 1) : (i == r ? 2.0f : -1.0f);
        lut[e] = make_float4(v[0], v[1], v[2], v[3]);
    }
}

// sp_observe with the 4-cell table, for L == LMAX (the ray cells of a launch
// written without per-cell compares or branches)
template <int LMAX>
__device__ __forceinline__ void sl_observe(const Params &p, const SPlanes &pl, Agent &g, const SRows &w, float *row,
                                           const float4 *clut) {
    const bool slow = (g.move_mask & 1u) || ((w.rec.y >> 17) & 1u);
    if (__builtin_expect(__ballot(slow) != 0ull || p.L != LMAX, 0)) {
        sb_observe<LMAX>(p, pl, g, w, row);
        return;
    }
    constexpr int L = LMAX;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
        const uint32_t e8 = ray_e8(w.rec, j);
        const int n = (int)(e8 & 0x7fu);
        const int m = n < L ? n : L;
        uint32_t t;   // bit s = the S bit of ray cell s + 1
        if (j == 0) t = (uint32_t)w.wx >> ((g.x + 1) & 31);
        else if (j == 2) t = (uint32_t)w.wy >> ((g.y + 1) & 31);
        else if (j == 4) t = w.wz >> ((g.z + 1) & 31);
        else if (j == 1) t = __builtin_bitreverse32((uint32_t)w.wx << ((32 - g.x) & 31));
        else if (j == 3) t = __builtin_bitreverse32((uint32_t)w.wy << ((32 - g.y) & 31));
        else t = __builtin_bitreverse32(w.wz << ((32 - g.z) & 31));
        const int slot = obs_slot(j, g.facing);
        float *out = row + slot * L;
#pragma unroll
        for (int c = 0; c < (L + 3) / 4; ++c) {
            const int r = min(max(m - 4 * c, -1), 4);
            const float4 q = clut[((t >> (4 * c)) & 15u) | ((uint32_t)(r + 1) << 4)];
            out[4 * c] = q.x;
            if (4 * c + 1 < L) out[4 * c + 1] = q.y;
            if (4 * c + 2 < L) out[4 * c + 2] = q.z;
            if (4 * c + 3 < L) out[4 * c + 3] = q.w;
        }
        row[6 * L + slot] = (float)m * 0.25f;   // round(count * 0.25, 2) is exact
    }
    row[6 * L + 6] = (float)g.last_action;
}

__device__ __forceinline__ void sb_load_rows(const Params &p, const SPlanes &pl, const Agent &g, const Room &R,
                                             SRows &w) {
    w.wx = pl.sx[g.y * p.ph + g.z];
    w.wy = pl.sy[g.x * p.ph + g.z];
    w.wz = pl.sz[g.x * p.pd + g.y];
    w.rec = p.rays[R.ray_off + (uint32_t)((g.x * R.D + g.y) * R.H + g.z)];
}

// after a move along axis ax the S word along that axis is the same row (only
// this agent writes it, so the cached copy is current): reload the other two
__device__ __forceinline__ void sb_move_rows(const Params &p, const SPlanes &pl, const Agent &g, const Room &R,
                                             SRows &w, int ax) {
    if (ax != 0) w.wx = pl.sx[g.y * p.ph + g.z];
    if (ax != 1) w.wy = pl.sy[g.x * p.ph + g.z];
    if (ax != 2) w.wz = pl.sz[g.x * p.pd + g.y];
    w.rec = p.rays[R.ray_off + (uint32_t)((g.x * R.D + g.y) * R.H + g.z)];
}

// reset for the lanes with `need` (as simple_reset_wave): the wave zeroes
// every resetting agent's planes, then each marks its start cell and senses.
template <int LMAX>
__device__ __forceinline__ void sb_reset_wave(const Params &p, const SPlanes &pl, bool need, uint32_t seed, Agent &g, uint32_t &goal,
                              Room &R, SRows &w, float *row, int lane, int block_agent0) {
    uint2 drawn = make_uint2(0u, 0u);
    if (need) drawn = simple_draw(p.envc, seed);
    uint64_t m = __ballot(need);
    const uint32_t n16 = p.agent_bytes >> 4;
    while (m) {
        const int src = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        uint4 *base = reinterpret_cast<uint4 *>(p.belief + (size_t)(block_agent0 + src) * p.agent_bytes);
        for (uint32_t q = (uint32_t)lane; q < n16; q += 64u) base[q] = make_uint4(0u, 0u, 0u, 0u);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (need) {
        g.room = (int)(drawn.x >> 24);
        R = load_room(p, g.room);
        g.x = drawn.x & 0xff;
        g.y = (drawn.x >> 8) & 0xff;
        g.z = (drawn.x >> 16) & 0xff;
        goal = drawn.y;
        g.facing = 0;
        g.last_action = 0;
        g.done = g.last_bump = g.near_wall = g.was_near_wall = false;
        g.step_count = 0;
        g.visited = 1;
        g.bumps = 0;
        g.cid = 0;
        g.move_mask = 0;
        w.wx = 1ull << g.x;                                                     // :86
        w.wy = 1ull << g.y;
        w.wz = 1u << g.z;
        if (p.sline) {                   // line layout: u32 SX[y][z], SY[x][z] (simple_line_kernel)
            reinterpret_cast<uint32_t *>(pl.sx)[g.y * p.ph + g.z] = (uint32_t)w.wx;
            reinterpret_cast<uint32_t *>(pl.sy)[g.x * p.ph + g.z] = (uint32_t)w.wy;
        } else {
            pl.sx[g.y * p.ph + g.z] = w.wx;
            pl.sy[g.x * p.ph + g.z] = w.wy;
            pl.sz[g.x * p.pd + g.y] = w.wz;
        }
        w.rec = p.rays[R.ray_off + (uint32_t)((g.x * R.D + g.y) * R.H + g.z)];
        sb_observe<LMAX>(p, pl, g, w, row);
    }
}

#ifndef VN_SIMPLE_PROF
#define VN_SIMPLE_PROF 0   // diagnostics build: per-section shader-clock totals (vn_debug_simple_prof)
#endif
#if VN_SIMPLE_PROF
__device__ unsigned long long g_simple_prof[16];
#define SB_T(k)                                                    \
    do {                                                           \
        const uint64_t t_ = __builtin_amdgcn_s_memtime();          \
        prof[k] += t_ - tprev;                                     \
        tprev = t_;                                                \
    } while (0)
#else
#define SB_T(k) \
    do {        \
    } while (0)
#endif

// vn_reset for the bit-plane layouts (line and word): 64 agents per block,
// one lane each -- the draws, the cleared planes, the start cell and the
// first observation, then the next episode's draw ahead for the step kernels
// (sp_reset_wave / sl_reset_wave).
template <int LMAX>
__global__ __launch_bounds__(64) void simple_bits_reset_kernel(Params p) {
    extern __shared__ float sstage[];   // [64][obs_dim]
    const int lane = threadIdx.x;
    const int a0 = blockIdx.x * 64;
    const int ai = a0 + lane;
    const bool live = ai < p.N;
    const int OD = p.obs_dim;
    float *row = sstage + lane * OD;
    const SPlanes pl = splanes(p, live ? ai : a0);
    Agent g = unpack(live ? p.hot[ai] : make_uint4(0u, 0u, 0u, 0u));
    uint32_t goal = live ? p.goal[ai] : 0u;
    Room R = load_room(p, g.room);
    SRows w;
    w.wx = w.wy = 0;
    w.wz = 0;
    w.rec = make_uint2(0u, 0u);
    const bool need = live && (!p.mask || p.mask[ai]);
    const uint32_t seed = need ? (uint32_t)p.seeds[ai] : 0u;
    sb_reset_wave<LMAX>(p, pl, need, seed, g, goal, R, w, row, lane, a0);
    if (need) {
        float *o = p.obs + (size_t)ai * OD;
        for (int k = 0; k < OD; ++k) o[k] = row[k];
        p.hot[ai] = pack(g);
        p.goal[ai] = goal;
        p.next_seed[ai] = seed + p.seed_stride;   // modulo 2^32
    }
    // the next episode's draw ahead (simple_pipe_kernel's sp_reset_wave)
    if (__ballot(need)) {
        const uint32_t s2 = seed + p.seed_stride;
        const uint2 d = need ? simple_draw(p.envc, s2) : make_uint2(0u, 0u);
        if (need) p.predraw[ai] = make_uint4(d.x, d.y, s2, 1u);
    }
}

// ----------------------------------------------------------------------------
// The bit-plane step with a store wave: block = 2 waves, wave 0 steps 64
// agents and stages each step's obs rows, rewards and flags in LDS (double
// buffered), wave 1 writes step k's staging to HBM while wave 0 computes step
// k+1.  vmcnt retires in issue order per wave, so in the one-wave kernel every
// step's loads waited for the previous step's ~8 obs stores per lane to
// complete; here the stepping wave issues no output stores at all (only its
// own S-word / Q updates).  One barrier per step hands a buffer over: the
// store wave has drained its LDS reads of buffer k&1 before it reaches the
// barrier after which wave 0 overwrites that buffer (step k+2).
// LDS: stage[2][64][OD] f32, reward[2][64] f32, flags[2][64] u32.
// ----------------------------------------------------------------------------
// Block barrier that orders only LDS: lgkmcnt(0) then s_barrier.  The store
// wave's HBM stores stay in flight across it (a __syncthreads() would wait
// vmcnt(0), i.e. for every store of the step to complete, before the
// stepping wave may go on).
#ifndef VN_LDS_BARRIER
#define VN_LDS_BARRIER 1
#endif
__device__ __forceinline__ void lds_handoff() {
#if VN_LDS_BARRIER
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);          // lgkmcnt(0) alone
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
#else
    __syncthreads();
#endif
}


// ----------------------------------------------------------------------------
// The bit-plane step with a store wave, software-pipelined by one step
// (the default simpleEnv kernel for rooms <= 64 x 64 x 31).  A step's move
// needs only the ray record of the agent's cell, which the previous step
// loaded, so the move of step k+1 is computed -- and the loads at its target
// cell (ray record, the two S words not along the move axis) issued --
// BEFORE step k's observation is built.  Those loads then land while step k
// observes; one stepping wave per SIMD no longer waits a full load round trip
// per step.  The pending move (action, direction, facing, target) is committed
// at the start of the next iteration (visit / S marks in the reference's
// order, :109-150); an auto-reset recomputes it from the start cell.  The
// stepping wave issues no output stores (the store wave does), so waiting for
// its loads never waits for obs stores.
// ----------------------------------------------------------------------------
// reset of the lanes with `need` for simple_pipe_kernel: as sb_reset_wave,
// but the MT19937 draw (a ~1.2k-step serial chain, ~15 us) is shared.  A
// lane's draw for its next episode seed is kept in nd = {start | room << 24,
// goal, seed, valid}.  A resetting lane whose nd is for its seed uses it; when
// any resetting lane has none, the wave runs the chain once for EVERY live
// lane (same instructions, so the same time as for one lane): the resetting
// lanes take their draw and the others keep theirs for their next reset.
// Measured: the chain was half of the kernel's time (resets ablated: 2x).
__device__ __forceinline__ uint2 sp_reset_draw(const Params &p, bool need, bool live, uint32_t seed, int lane, uint4 &nd,
                                               uint32_t *mt_lds) {
    const bool have = need && nd.w == 1u && nd.z == seed;
    uint2 drawn = have ? make_uint2(nd.x, nd.y) : make_uint2(0u, 0u);
    if (need) nd.w = 0u;                                   // consumed: the next episode has another seed
    if (__ballot(need && !have)) {
        // one chain pass for the wave: a resetting lane without a draw computes
        // this episode's; one with a draw the episode after it (seed + stride);
        // the others their next episode's if they have none
        const uint32_t s2 = (need && have) ? seed + p.seed_stride : seed;
        mt_outputs_wide(s2, mt_lds + lane * MT_WS);
        MtLdsStream mt;
        mt.row = mt_lds + lane * MT_WS;
        mt.seed = s2;
        mt.used = 0;
        mt.err = p.envc->err;
        const uint2 d2 = live ? simple_draw_from(p.envc, mt) : make_uint2(0u, 0u);
        if (need && !have) drawn = d2;
        else if (live) nd = make_uint4(d2.x, d2.y, s2, 1u);
    }
    return drawn;
}

template <int LMAX>
__device__ __forceinline__ void sp_reset_wave(const Params &p, const SPlanes &pl, bool need, bool live, uint32_t seed,
                                              Agent &g, uint32_t &goal, Room &R, SRows &w, float *row, int lane,
                                              int block_agent0, uint4 &nd, uint32_t *mt_lds) {
    const uint2 drawn = sp_reset_draw(p, need, live, seed, lane, nd, mt_lds);
    uint64_t m = __ballot(need);
    const uint32_t n16 = p.agent_bytes >> 4;
    while (m) {
        const int src = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        uint4 *base = reinterpret_cast<uint4 *>(p.belief + (size_t)(block_agent0 + src) * p.agent_bytes);
        for (uint32_t q = (uint32_t)lane; q < n16; q += 64u) base[q] = make_uint4(0u, 0u, 0u, 0u);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (need) {
        g.room = (int)(drawn.x >> 24);
        R = load_room(p, g.room);
        g.x = drawn.x & 0xff;
        g.y = (drawn.x >> 8) & 0xff;
        g.z = (drawn.x >> 16) & 0xff;
        goal = drawn.y;
        g.facing = 0;
        g.last_action = 0;
        g.done = g.last_bump = g.near_wall = g.was_near_wall = false;
        g.step_count = 0;
        g.visited = 1;
        g.bumps = 0;
        g.cid = 0;
        g.move_mask = 0;
        w.wx = 1ull << g.x;                                                     // :86
        w.wy = 1ull << g.y;
        w.wz = 1u << g.z;
        pl.sx[g.y * p.ph + g.z] = w.wx;
        pl.sy[g.x * p.ph + g.z] = w.wy;
        pl.sz[g.x * p.pd + g.y] = w.wz;
        w.rec = p.rays[R.ray_off + (uint32_t)((g.x * R.D + g.y) * R.H + g.z)];
        sb_observe<LMAX>(p, pl, g, w, row);
    }
}

struct SPend {
    int a, d, facing, nx, ny, nz;
    bool moved;
};

template <int LMAX, bool EXT>
__global__ __launch_bounds__(128) void simple_pipe_kernel(Params p) {
    extern __shared__ float sm[];
    const int OD = p.obs_dim, L = p.L;
    float *stage = sm;
    float *srew = sm + 2 * 64 * OD;
    uint32_t *sflg = reinterpret_cast<uint32_t *>(srew + 2 * 64);
    const int lane = threadIdx.x & 63;
    const int a0 = blockIdx.x * 64;
    const int rows = min(64, p.N - a0);

    if (threadIdx.x >= 64) {                     // ---- store wave (as simple_split_kernel) ----
        for (int k = 0; k < p.K; ++k) {
            lds_handoff();                     // step k staged in buffer k & 1
            const int b = k & 1;
            const float *st = stage + b * 64 * OD;
            float *dst = p.obs + ((size_t)k * p.N + a0) * OD;
            if (VN_ABLATE & 16u) {
            } else if (!((rows * OD) & 3) && !(reinterpret_cast<uintptr_t>(dst) & 15u)) {
                const float4 *s4 = reinterpret_cast<const float4 *>(st);
                float4 *d4 = reinterpret_cast<float4 *>(dst);
                for (int q = lane; q < (rows * OD) >> 2; q += 64) obs_store(d4 + q, s4[q]);
            } else {
                for (int q = lane; q < rows * OD; q += 64) __builtin_nontemporal_store(st[q], dst + q);
            }
            if (lane < rows) {
                const size_t o = (size_t)k * p.N + a0 + lane;
                const uint32_t f = sflg[b * 64 + lane];
                if (p.reward) p.reward[o] = srew[b * 64 + lane];
                if (p.term) p.term[o] = (uint8_t)(f & 1u);
                if (p.trunc) p.trunc[o] = (uint8_t)(f >> 1);
            }
        }
        return;
    }

    // ---- stepping wave ----
    // Every global store of the step loop is issued unconditionally (the
    // evicted S words go through a buffer resource over the block's belief
    // maps; a lane with nothing to store gives an out-of-range offset, which
    // the hardware drops).  vmcnt retires in issue order, so a load can be
    // waited for with the stores issued after it still in flight only when
    // their count is the same on every path; a store skipped by a branch
    // made hipcc wait vmcnt(0) -- for the stores too -- in every step.
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
        p.belief + (size_t)a0 * p.agent_bytes, 0, (int)((uint32_t)rows * p.agent_bytes), 0x00020000);
    const uint32_t lane_off = (uint32_t)lane * p.agent_bytes;
    const int ai = a0 + lane;
    const bool live = ai < p.N;
    const SPlanes pl = splanes(p, live ? ai : a0);
    Agent g = unpack(live ? p.hot[ai] : make_uint4(0u, 0u, 0u, 0u));
    uint32_t goal = live ? p.goal[ai] : 0u;
    uint32_t next_seed = live ? p.next_seed[ai] : 0u;
    uint4 nd = live ? p.predraw[ai] : make_uint4(0u, 0u, 0u, 0u);   // draw ahead (sp_reset_wave)
    Room R = load_room(p, g.room);
    SRows w;                                     // S words + ray record at the agent's (committed) cell
    w.wx = w.wy = 0;
    w.wz = 0;
    w.rec = make_uint2(0u, 0u);
    if (live) sb_load_rows(p, pl, g, R, w);
    vn_touch(w.wx);
    vn_touch(w.wy);
    vn_touch(w.wz);
    vn_touch(w.rec.x);
    vn_touch(w.rec.y);
    vn_touch((uint32_t)R.ray_off);
    vn_touch((uint32_t)R.total_free);
    vn_touch((uint32_t)(R.D | (R.H << 8)));

    uint4 r4 = make_uint4(0u, 0u, 0u, 0u);      // Philox block r4blk (4 steps)
    uint64_t r4blk = ~0ull;
    SPend pm;                                    // the pending move
    SRows wn;                                    // ... and the rows at its target (in flight)
    uint64_t cbx = 0ull, cby = 0ull;             // S bits its commit adds to wn's kept rows
    uint32_t cbz = 0u;
    // The S words in w are write-back cached: a mark sets their dirty bits
    // (1 x, 2 y, 4 z); a word is stored when a move replaces it (eviction:
    // its row at the cell being left) and at the end of the launch.  The
    // evicted words of a commit are stored after the next move's loads; a
    // load of an evicted row takes the evicted value (forwarding).
    uint32_t sdirty = 0u, evm = 0u;              // dirty words; evicted words pending store
    uint64_t evx = 0ull, evy = 0ull;             // evicted values ...
    uint32_t evz = 0u;
    int evyx = 0, evxy = 0, evz_ = 0, evxx = 0, evyy = 0;   // ... and their rows: x (y,z)  y (x,z)  z (x,y)
    // the move of launch step k from the committed state; issues the target's loads
    auto premove = [&](int k) {
        const uint64_t t = p.t0 + (uint64_t)k;
        int a;
        if (EXT) {
            a = p.actions[(size_t)k * p.N + (live ? ai : a0)];
        } else {
            if ((t >> 2) != r4blk) {
                r4blk = t >> 2;
                r4 = philox4x32_10(p.policy_seed, p.gid_base + (uint64_t)(live ? ai : a0), t >> 2);
            }
            const uint32_t word = (t & 3) == 0 ? r4.x : (t & 3) == 1 ? r4.y : (t & 3) == 2 ? r4.z : r4.w;
            a = (int)(((uint64_t)word * 6u) >> 32);
        }
        const int d = a < 4 ? rel_dir(a, g.facing) : (a == 4 ? 4 : 5);
        pm.a = a;
        pm.d = d;
        pm.facing = a < 4 ? facing_of(d) : g.facing;                 // :164-171
        pm.moved = (ray_e8(w.rec, d) & 0x7fu) >= 1u;
        pm.nx = g.x + (pm.moved ? (d == 0 ? 1 : d == 1 ? -1 : 0) : 0);
        pm.ny = g.y + (pm.moved ? (d == 2 ? 1 : d == 3 ? -1 : 0) : 0);
        pm.nz = g.z + (pm.moved ? (d == 4 ? 1 : d == 5 ? -1 : 0) : 0);
        wn = w;
        if (pm.moved) {
            // the S word along the move axis is the same row (kept); the other two
            // rows and the ray record are the target's.  These rows never hold
            // the bit the commit of this move sets (they are off the current cell).
            const int ax = d >> 1;
            if (ax != 0) wn.wx = ((evm & 1u) && evyx == pm.ny && evz_ == pm.nz) ? evx : pl.sx[pm.ny * p.ph + pm.nz];
            if (ax != 1) wn.wy = ((evm & 2u) && evxy == pm.nx && evz_ == pm.nz) ? evy : pl.sy[pm.nx * p.ph + pm.nz];
            if (ax != 2) wn.wz = ((evm & 4u) && evxx == pm.nx && evyy == pm.ny) ? evz : pl.sz[pm.nx * p.pd + pm.ny];
            wn.rec = p.rays[R.ray_off + (uint32_t)((pm.nx * R.D + pm.ny) * R.H + pm.nz)];
        }
    };
    if (live && p.K > 0) premove(0);
#if VN_SIMPLE_PROF
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tprev = __builtin_amdgcn_s_memtime();
#endif

    for (int k = 0; k < p.K; ++k) {
        const int b = k & 1;
        float *row = stage + b * 64 * OD + lane * OD;
        bool trunc = false, term = false;
        int a = 0;
        bool moved = false, explored = false, seen = true;
        if (live) {
            // ---- commit step k (:109-150) ----
            if (p.actions_out) p.actions_out[(size_t)k * p.N + ai] = pm.a;
            g.step_count += 1;
            trunc = g.step_count >= R.total_free;                      // :111, max_steps = total_free (:409)
            g.facing = pm.facing;
            a = pm.a;
            moved = pm.moved;
            if (moved) {                                                 // _mark_visited (:273-298)
                const int ax = pm.d >> 1;
                // the target's S bit from the cached word of the move axis (kept in wn)
                seen = ax == 0 ? ((w.wx >> pm.nx) & 1ull) : ax == 1 ? ((w.wy >> pm.ny) & 1ull) : ((w.wz >> pm.nz) & 1u);
                // evict the dirty words this move replaces (rows at the cell left)
                evm = sdirty & ~(1u << ax);
                evx = w.wx;
                evy = w.wy;
                evz = w.wz;
                evyx = g.y;
                evz_ = g.z;
                evxy = g.x;
                evxx = g.x;
                evyy = g.y;
                sdirty &= 1u << ax;
                g.x = pm.nx;
                g.y = pm.ny;
                g.z = pm.nz;
                w = wn;
            } else {
                evm = 0u;
            }
            // the bits of the previous step's mark that this move's rows were
            // copied without (see below)
            w.wx |= cbx;
            w.wy |= cby;
            w.wz |= cbz;
            cbx = cby = 0ull;
            cbz = 0u;
            g.last_action = a;                                           // :137
            SB_T(0);
            // ---- the next step's move and its loads, issued before this step's
            // S-mark stores (a wait for these loads then never waits for them) ----
            if (k + 1 < p.K) premove(k + 1);
            if (!(VN_ABLATE & 1024u)) {                 // the evicted words, behind the loads
                constexpr uint32_t OFF = 0x80000000u;   // out of range: dropped
                typedef uint32_t u32x2_t __attribute__((ext_vector_type(2)));
                const u32x2_t vx = {(uint32_t)evx, (uint32_t)(evx >> 32)}, vy = {(uint32_t)evy, (uint32_t)(evy >> 32)};
                __builtin_amdgcn_raw_buffer_store_b64(
                    vx, brs, (evm & 1u) ? lane_off + 8u * (uint32_t)(evyx * p.ph + evz_) : OFF, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b64(
                    vy, brs, (evm & 2u) ? lane_off + p.sy_off + 8u * (uint32_t)(evxy * p.ph + evz_) : OFF, 0, 0);
                __builtin_amdgcn_raw_buffer_store_b32(
                    evz, brs, (evm & 4u) ? lane_off + p.sz_off + 4u * (uint32_t)(evxx * p.pd + evyy) : OFF, 0, 0);
            }
            evm = 0u;
            SB_T(1);
            if (moved) {
                // a Q cell (internal_grid 2) is entered without counting, but it
                // is a sensing position all the same, so S is set
                const bool q = (g.move_mask & 1u) && ((pl.qz[g.x * p.pd + g.y] >> g.z) & 1u);
                if (!seen) {
                    const uint64_t bx = 1ull << g.x, by = 1ull << g.y;
                    const uint32_t bz = 1u << g.z;
                    w.wx |= bx;
                    w.wy |= by;
                    w.wz |= bz;
                    // the pending move copied its kept row(s) from w before this
                    // mark (all three if it does not move): carried into its
                    // commit (wn itself is the target of loads in flight)
                    const int nax = pm.moved ? pm.d >> 1 : -1;
                    if (nax <= 0) cbx = bx;
                    if (nax == -1 || nax == 1) cby = by;
                    if (nax == -1 || nax == 2) cbz = bz;
                    sdirty = 7u;
                    if (!q) {
                        g.visited += 1;
                        explored = true;
                    }
                }
            }
            SB_T(2);
            if (!(VN_ABLATE & 4u)) sp_observe<LMAX>(p, pl, g, w, row);   // :139
            SB_T(3);
            // compute_reward (:189-217), f64 in the reference's order
            double r = -0.1;
            if (!moved) {
                g.bumps += 1;
                r += -10.0;
            }
            if (a != 2 && a < 4) r += 0.05;
            const int gx = goal & 0xff, gy = (goal >> 8) & 0xff, gz = (goal >> 16) & 0xff;
            if (g.x == gx && g.y == gy && g.z >= gz && g.z - gz < 5) {   // SPOT_GOAL_HEIGTH = 5 (:201-206)
                g.done = true;
                r += 100.0;
            }
            if (trunc) r += 0.0;
            if (explored) r += 1.0;
            term = g.done;
            const size_t o = (size_t)k * p.N + ai;
            srew[b * 64 + lane] = (float)r;
            sflg[b * 64 + lane] = (term ? 1u : 0u) | (trunc ? 2u : 0u);
            if (p.reward64) p.reward64[o] = r;
            if ((term || trunc) && p.autoreset && p.terminal_obs) {
                float *to = p.terminal_obs + o * OD;
                for (int q = 0; q < OD; ++q) to[q] = row[q];
            }
        }
        SB_T(4);
        // SB3 VecEnv auto-reset
        const bool need = live && p.autoreset && (term || trunc) && !(VN_ABLATE & 512u);
        if (__ballot(need)) {
            sp_reset_wave<LMAX>(p, pl, need, live, next_seed, g, goal, R, w, row, lane, a0, nd,
                                reinterpret_cast<uint32_t *>(sflg + 2 * 64));
            if (need) {
                next_seed += p.seed_stride;
                cbx = cby = 0ull;
                cbz = 0u;
                sdirty = 0u;                             // the reset stored the start cell's words
                evm = 0u;
                if (k + 1 < p.K) premove(k + 1);                         // from the start cell
                vn_touch(w.rec.x);
                vn_touch(w.rec.y);
                vn_touch((uint32_t)R.ray_off);
                vn_touch((uint32_t)R.total_free);
                vn_touch((uint32_t)(R.D | (R.H << 8)));
            }
        }
        SB_T(5);
        lds_handoff();                         // hand buffer b to the store wave
        SB_T(6);
    }
#if VN_SIMPLE_PROF
    if (lane == 0) {
        uint64_t tot = 0;
        for (int q = 0; q < 7; ++q) {
            atomicAdd(&g_simple_prof[q], (unsigned long long)prof[q]);
            tot += prof[q];
        }
        atomicAdd(&g_simple_prof[7], tot);
        atomicAdd(&g_simple_prof[8], 1ull);
    }
#endif
    if (live) {
        if (sdirty & 1u) pl.sx[g.y * p.ph + g.z] = w.wx;
        if (sdirty & 2u) pl.sy[g.x * p.ph + g.z] = w.wy;
        if (sdirty & 4u) pl.sz[g.x * p.pd + g.y] = w.wz;
        p.hot[ai] = pack(g);
        p.goal[ai] = goal;
        p.next_seed[ai] = next_seed;
        p.predraw[ai] = nd;
    }
    (void)L;
}


// ============================================================================
// simpleEnv, line layout (the default for rooms up to 32 x 32 x 8, e.g. the
// bench's 32x32x8 box).  Same belief as the bit-plane layout -- S (cells
// stood on) and Q (edge-quirk marks), every other internal_grid value derived
// -- but S is kept as LINES: SX[y] = 8 u32 words over z (bit x), SY[x] = 8 u32
// words over z (bit y), 32 B each; a column's z bits (the up / down rays) are
// bit x of the SX[y] line, so there is no third copy.  The stepping lane keeps
// the two lines through its cell in LDS: a move along x replaces the SY line,
// along y the SX line, along z neither; the line left is stored back if it
// was marked.
// Why (rocprofv3, round 3): the simpleEnv step is bound by the CUs' 64-B
// request rate -- the address unit is busy 87-95 % of the kernel, at 5.7
// requests per env-step, 1.1 of them the evicted S words of the word layout
// (each move replaced 2-3 words; without those stores the kernel ran 1.4x).
// A lane's 32-B line access is 2 x 16 B; lane pairs split it so that both
// halves of one line go out in ONE instruction (a request per line, not per
// half): instruction 1 moves the even lane's line, instruction 2 the odd
// lane's, and the halves are swapped across the pair with one DPP move.
// Every line load / store is issued every step (an out-of-range buffer offset
// when a lane has none: no request, and the same vmcnt count on every path).
// LDS per lane: the X and Y line (12-word stride: 16-B aligned rows).
// QZ (edge-quirk marks) as in the bit-plane layout.
// ============================================================================
constexpr int SL_STRIDE = 12;   // words per LDS line slot
constexpr uint32_t SL_OFF = 0x80000000u;   // out-of-range buffer offset: dropped
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

struct SLine {
    u32x4_t h0, h1;   // words 0-3, 4-7
};

__device__ __forceinline__ uint32_t dpp_swap_pair(uint32_t v) {   // lane i <- lane i ^ 1
    return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);
}
__device__ __forceinline__ u32x4_t dpp_swap_pair4(u32x4_t v) {
    u32x4_t r;
    r.x = dpp_swap_pair(v.x);
    r.y = dpp_swap_pair(v.y);
    r.z = dpp_swap_pair(v.z);
    r.w = dpp_swap_pair(v.w);
    return r;
}

// lane-pair line load: each lane gets the line at its byte offset `off`
// (SL_OFF: none, zeros).  Issue and finish (the swap across the pair, which
// needs the data) are split so the loads stay in flight across a step.  Both
// must run with the whole wave active.
__device__ __forceinline__ SLine sl_pair_issue(__amdgpu_buffer_rsrc_t rs, uint32_t off, bool odd) {
    const uint32_t off_p = dpp_swap_pair(off);
    const uint32_t ae = odd ? off_p : off, ao = odd ? off : off_p;     // the pair's even / odd line
    const uint32_t half = odd ? 16u : 0u;
    SLine r;   // even: h0 = own h0, h1 = partner's h0; odd: h0 = partner's h1, h1 = own h1
    r.h0 = __builtin_amdgcn_raw_buffer_load_b128(rs, ae == SL_OFF ? SL_OFF : ae + half, 0, 0);
    r.h1 = __builtin_amdgcn_raw_buffer_load_b128(rs, ao == SL_OFF ? SL_OFF : ao + half, 0, 0);
    return r;
}
__device__ __forceinline__ SLine sl_pair_finish(const SLine &r, bool odd) {
    const u32x4_t sw = dpp_swap_pair4(odd ? r.h0 : r.h1);
    SLine l;
    l.h0 = odd ? sw : r.h0;
    l.h1 = odd ? r.h1 : sw;
    return l;
}
__device__ __forceinline__ SLine sl_pair_load(__amdgpu_buffer_rsrc_t rs, uint32_t off, bool odd) {
    return sl_pair_finish(sl_pair_issue(rs, off, odd), odd);
}

// lane-pair line store of each lane's line `l` at `off` (SL_OFF: none)
__device__ __forceinline__ void sl_pair_store(__amdgpu_buffer_rsrc_t rs, uint32_t off, const SLine &l, bool odd) {
    const uint32_t off_p = dpp_swap_pair(off);
    const uint32_t ae = odd ? off_p : off, ao = odd ? off : off_p;
    const uint32_t half = odd ? 16u : 0u;
    const u32x4_t sw = dpp_swap_pair4(odd ? l.h0 : l.h1);   // even gets the odd lane's h0, odd the even's h1
    __builtin_amdgcn_raw_buffer_store_b128(odd ? sw : l.h0, rs, ae == SL_OFF ? SL_OFF : ae + half, 0, 0);
    __builtin_amdgcn_raw_buffer_store_b128(odd ? l.h1 : sw, rs, ao == SL_OFF ? SL_OFF : ao + half, 0, 0);
}

__device__ __forceinline__ void sl_lds_put(uint32_t *slot, const SLine &l) {
    reinterpret_cast<u32x4_t *>(slot)[0] = l.h0;
    reinterpret_cast<u32x4_t *>(slot)[1] = l.h1;
}
__device__ __forceinline__ SLine sl_lds_get(const uint32_t *slot) {
    SLine l;
    l.h0 = reinterpret_cast<const u32x4_t *>(slot)[0];
    l.h1 = reinterpret_cast<const u32x4_t *>(slot)[1];
    return l;
}
// bit z = bit b of word z (the column's S bits from the SX line)
__device__ __forceinline__ uint32_t sl_column(const SLine &l, int b) {
    const uint32_t w[8] = {l.h0.x, l.h0.y, l.h0.z, l.h0.w, l.h1.x, l.h1.y, l.h1.z, l.h1.w};
    uint32_t c = 0;
#pragma unroll
    for (int z = 0; z < 8; ++z) c |= ((w[z] >> b) & 1u) << z;
    return c;
}

// reset of the lanes with `need` (sp_reset_wave in the line layout): the
// wave zeroes every resetting agent's SX / SY lines (and QZ if it holds
// marks), then each marks its start cell in its LDS lines (dirty) and senses
template <int LMAX>
__device__ __forceinline__ void sl_reset_wave(const Params &p, const SPlanes &pl, bool need, bool live, uint32_t seed,
                                              Agent &g, uint32_t &goal, Room &R, SRows &w, float *row, int lane,
                                              int block_agent0, uint4 &nd, uint32_t *mt_lds, uint32_t *lx,
                                              uint32_t *ly) {
    const uint2 drawn = sp_reset_draw(p, need, live, seed, lane, nd, mt_lds);
    const bool hadq = need && (g.move_mask & 1u);
    uint64_t m = __ballot(need);
    const uint64_t mq = __ballot(hadq);
    while (m) {
        const int src = __ffsll((unsigned long long)m) - 1;
        m &= m - 1;
        // QZ (at the end of the agent's block) is all zero unless the episode marked it
        const uint32_t n16 = (((mq >> src) & 1ull) ? p.agent_bytes : p.qz_off) >> 4;
        uint4 *base = reinterpret_cast<uint4 *>(p.belief + (size_t)(block_agent0 + src) * p.agent_bytes);
        for (uint32_t q = (uint32_t)lane; q < n16; q += 64u) base[q] = make_uint4(0u, 0u, 0u, 0u);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    if (need) {
        g.room = (int)(drawn.x >> 24);
        R = load_room(p, g.room);
        g.x = drawn.x & 0xff;
        g.y = (drawn.x >> 8) & 0xff;
        g.z = (drawn.x >> 16) & 0xff;
        goal = drawn.y;
        g.facing = 0;
        g.last_action = 0;
        g.done = g.last_bump = g.near_wall = g.was_near_wall = false;
        g.step_count = 0;
        g.visited = 1;
        g.bumps = 0;
        g.cid = 0;
        g.move_mask = 0;
        w.wx = 1ull << g.x;                                                     // :86
        w.wy = 1ull << g.y;
        w.wz = 1u << g.z;
#pragma unroll
        for (int z = 0; z < 8; ++z) {
            lx[z] = z == g.z ? (uint32_t)w.wx : 0u;
            ly[z] = z == g.z ? (uint32_t)w.wy : 0u;
        }
        w.rec = p.rays[R.ray_off + (uint32_t)((g.x * R.D + g.y) * R.H + g.z)];
        sb_observe<LMAX>(p, pl, g, w, row);
    }
}

template <int LMAX, bool EXT>
__global__ __launch_bounds__(128) void simple_line_kernel(Params p) {
    extern __shared__ float sm[];
    const int OD = p.obs_dim, L = p.L;
    float *stage = sm;
    float *srew = sm + 2 * 64 * OD;
    uint32_t *sflg = reinterpret_cast<uint32_t *>(srew + 2 * 64);
    uint32_t *mt_lds = sflg + 2 * 64;
    uint32_t *lines = mt_lds + 64 * MT_WS + 4;   // [3][64][SL_STRIDE] (X, Y, dummy); 16-B aligned
    float4 *clut = reinterpret_cast<float4 *>(lines + 3 * 64 * SL_STRIDE);   // [SL_CLUT] (sl_observe)
    float *srt = reinterpret_cast<float *>(clut + SL_CLUT);   // [16] f32, then [16] f64 rewards (TAB_SREW)
    const double *srt64 = reinterpret_cast<const double *>(srt + 16);
    const int lane = threadIdx.x & 63;
    const int a0 = blockIdx.x * 64;
    const int rows = min(64, p.N - a0);

    if (threadIdx.x >= 64) {                     // ---- store wave (as simple_pipe_kernel) ----
        for (int k = 0; k < p.K; ++k) {
            lds_handoff();                     // step k staged in buffer k & 1
            const int b = k & 1;
            const float *st = stage + b * 64 * OD;
            float *dst = p.obs + ((size_t)k * p.N + a0) * OD;
            if (VN_ABLATE & 16u) {
            } else if (!((rows * OD) & 3) && !(reinterpret_cast<uintptr_t>(dst) & 15u)) {
                const float4 *s4 = reinterpret_cast<const float4 *>(st);
                float4 *d4 = reinterpret_cast<float4 *>(dst);
                for (int q = lane; q < (rows * OD) >> 2; q += 64) obs_store(d4 + q, s4[q]);
            } else {
                for (int q = lane; q < rows * OD; q += 64) __builtin_nontemporal_store(st[q], dst + q);
            }
            if (lane < rows) {
                const size_t o = (size_t)k * p.N + a0 + lane;
                const uint32_t f = sflg[b * 64 + lane];
                if (p.reward) p.reward[o] = srew[b * 64 + lane];
                if (p.term) p.term[o] = (uint8_t)(f & 1u);
                if (p.trunc) p.trunc[o] = (uint8_t)(f >> 1);
            }
        }
        return;
    }

    // ---- stepping wave ----
    const __amdgpu_buffer_rsrc_t brs = __builtin_amdgcn_make_buffer_rsrc(
        p.belief + (size_t)a0 * p.agent_bytes, 0, (int)((uint32_t)rows * p.agent_bytes), 0x00020000);
    const uint32_t lane_off = (uint32_t)lane * p.agent_bytes;
    const bool odd = lane & 1;
    const int ai = a0 + lane;
    const bool live = ai < p.N;
    uint32_t *lx = lines + lane * SL_STRIDE;           // SX[g.y]
    uint32_t *ly = lines + (64 + lane) * SL_STRIDE;    // SY[g.x]
    uint32_t *lz = lines + (128 + lane) * SL_STRIDE;   // target of a commit's line write without a line
    sl_build_cell_lut(clut, lane);
    if (lane < 48) srt[lane] = p.lut[TAB_SREW + lane];
    const SPlanes pl = splanes(p, live ? ai : a0);
    Agent g = unpack(live ? p.hot[ai] : make_uint4(0u, 0u, 0u, 0u));
    uint32_t goal = live ? p.goal[ai] : 0u;
    uint32_t next_seed = live ? p.next_seed[ai] : 0u;
    uint4 nd = live ? p.predraw[ai] : make_uint4(0u, 0u, 0u, 0u);   // draw ahead (sp_reset_wave)
    Room R = load_room(p, g.room);
    auto xline_off = [&](int y) { return lane_off + 32u * (uint32_t)y; };
    auto yline_off = [&](int x) { return lane_off + p.sy_off + 32u * (uint32_t)x; };
    SRows w;                                     // S words + ray record at the agent's (committed) cell
    {
        const SLine l0 = sl_pair_load(brs, live ? xline_off(g.y) : SL_OFF, odd);
        const SLine l1 = sl_pair_load(brs, live ? yline_off(g.x) : SL_OFF, odd);
        sl_lds_put(lx, l0);
        sl_lds_put(ly, l1);
        w.wx = lx[g.z & 7];
        w.wy = ly[g.z & 7];
        w.wz = sl_column(l0, g.x & 31);
        w.rec = live ? p.rays[R.ray_off + (uint32_t)((g.x * R.D + g.y) * R.H + g.z)] : make_uint2(0u, 0u);
    }
    vn_touch((uint32_t)R.ray_off);
    vn_touch((uint32_t)R.total_free);
    vn_touch((uint32_t)(R.D | (R.H << 8)));

    uint4 r4 = make_uint4(0u, 0u, 0u, 0u);      // Philox block r4blk (4 steps)
    uint64_t r4blk = ~0ull;
    SPend pm;                                    // the pending move ...
    SLine lr;                                    // ... the line it brings in (raw pair loads, in flight;
    bool lfwd = false;                           //     or the replaced line: lfwd) ...
    uint32_t lpend = SL_OFF;                     //     (its offset: a re-issue repeats it) ...
    uint2 rn = make_uint2(0u, 0u);               // ... and its target's ray record (in flight)
    uint32_t dirty = 0u;                         // 1: the LDS X line is marked, 2: the Y line
    SLine ev;                                    // the line the last commit replaced, stored after the
    uint32_t ev_off = SL_OFF;                    // next move's loads (a load of it takes it from here)
    ev.h0 = ev.h1 = u32x4_t{0u, 0u, 0u, 0u};
    lr = ev;
    // the move of launch step k from the committed state; issues the target's loads
    // keep: lanes without `act` keep their pending move.  The line loads are
    // re-issued for them too: a lane pair's two loads carry both lanes' lines
    // (sl_pair_issue), so the pair always issues together.
    auto premove = [&](int k, bool act, bool keep) {
        uint32_t loff = (keep && !act) ? lpend : SL_OFF;
        uint32_t rcell = 0u;
        if (act) {
            const uint64_t t = p.t0 + (uint64_t)k;
            int a;
            if (EXT) {
                a = p.actions[(size_t)k * p.N + ai];
            } else {
                if ((t >> 2) != r4blk) {
                    r4blk = t >> 2;
                    r4 = philox4x32_10(p.policy_seed, p.gid_base + (uint64_t)ai, t >> 2);
                }
                const uint32_t word = (t & 3) == 0 ? r4.x : (t & 3) == 1 ? r4.y : (t & 3) == 2 ? r4.z : r4.w;
                a = (int)(((uint64_t)word * 6u) >> 32);
            }
            const int d = a < 4 ? rel_dir(a, g.facing) : (a == 4 ? 4 : 5);
            pm.a = a;
            pm.d = d;
            pm.facing = a < 4 ? facing_of(d) : g.facing;                 // :164-171
            pm.moved = (ray_e8(w.rec, d) & 0x7fu) >= 1u;
            pm.nx = g.x + (pm.moved ? (d == 0 ? 1 : d == 1 ? -1 : 0) : 0);
            pm.ny = g.y + (pm.moved ? (d == 2 ? 1 : d == 3 ? -1 : 0) : 0);
            pm.nz = g.z + (pm.moved ? (d == 4 ? 1 : d == 5 ? -1 : 0) : 0);
            rcell = (uint32_t)((pm.nx * R.D + pm.ny) * R.H + pm.nz);
            // the line a move along x (y) brings in: SY[nx] (SX[ny]); from ev (no
            // request) if it is the line the last commit replaced
            if (pm.moved && d < 4) {
                const uint32_t o = d < 2 ? yline_off(pm.nx) : xline_off(pm.ny);
                if (o != ev_off) loff = o;
            }
        }
        lr = sl_pair_issue(brs, loff, odd);
        lpend = loff;
        const uint2 rc = p.rays[R.ray_off + rcell];
        if (!keep || act) {
            lfwd = loff == SL_OFF;               // forwarded from ev (or unused)
            rn = rc;
        }
    };
    if (p.K > 0) premove(0, live, false);
#if VN_SIMPLE_PROF
    uint64_t prof[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    uint64_t tprev = __builtin_amdgcn_s_memtime();
#endif

    for (int k = 0; k < p.K; ++k) {
        const int b = k & 1;
        float *row = stage + b * 64 * OD + lane * OD;
        bool trunc = false, term = false;
        int a = 0;
        bool moved = false, explored = false, seen = true;
        if (live) {
            // ---- commit step k (:109-150) ----
            if (p.actions_out) p.actions_out[(size_t)k * p.N + ai] = pm.a;
            g.step_count += 1;
            trunc = g.step_count >= R.total_free;                      // :111, max_steps = total_free (:409)
            g.facing = pm.facing;
            a = pm.a;
            moved = pm.moved;
        }
        {
            // _mark_visited (:273-298); straight-line for every lane: a lane
            // whose move brings no line writes it to its dummy slot
            const int ax = moved ? pm.d >> 1 : 3;
            const bool xy = ax < 2;
            // the target's S bit from the word along the move axis
            seen = !moved || (ax == 0 ? ((w.wx >> pm.nx) & 1ull) : ax == 1 ? ((w.wy >> pm.ny) & 1ull)
                                                                            : ((w.wz >> pm.nz) & 1u));
            // replace the line across the move axis: the old one is stored if marked
            uint32_t *slot = ax == 0 ? ly : ax == 1 ? lx : lz;
            const uint32_t dbit = ax == 0 ? 2u : 1u;
            const SLine lf = sl_pair_finish(lr, odd);
            const SLine ln = lfwd ? ev : lf;
            ev = sl_lds_get(slot);
            ev_off = (xy && (dirty & dbit)) ? (ax == 0 ? yline_off(g.x) : xline_off(g.y)) : SL_OFF;
            dirty &= xy ? ~dbit : ~0u;
            sl_lds_put(slot, ln);
            if (moved) {
                g.x = pm.nx;
                g.y = pm.ny;
                g.z = pm.nz;
                w.rec = rn;
            }
            w.wx = lx[g.z];
            w.wy = ly[g.z];
            const uint32_t col = sl_column(sl_lds_get(lx), g.x);
            if (xy) w.wz = col;
        }
        if (live) {
            g.last_action = a;                                           // :137
        }
        SB_T(0);
        // ---- the replaced line's store, then the next step's move and its
        // loads: vmcnt retires in issue order, so the wait for the loads (a
        // step later) covers the older store at no cost; a store issued after
        // them would be waited for as well (the compiler's counts do not
        // include stores on this target and it waits vmcnt(0) for the last load) ----
        sl_pair_store(brs, ev_off, ev, odd);
        premove(k + 1, live && k + 1 < p.K, false);
        ev_off = SL_OFF;
        SB_T(1);
        if (live) {
            if (moved) {
                // a Q cell (internal_grid 2) is entered without counting, but it
                // is a sensing position all the same, so S is set
                const bool q = (g.move_mask & 1u) && ((pl.qz[g.x * p.pd + g.y] >> g.z) & 1u);
                if (!seen) {
                    w.wx |= 1ull << g.x;
                    w.wy |= 1ull << g.y;
                    w.wz |= 1u << g.z;
                    lx[g.z] = (uint32_t)w.wx;
                    ly[g.z] = (uint32_t)w.wy;
                    dirty = 3u;
                    if (!q) {
                        g.visited += 1;
                        explored = true;
                    }
                }
            }
            SB_T(2);
            if (!(VN_ABLATE & 4u)) sl_observe<LMAX>(p, pl, g, w, row, clut);   // :139
            SB_T(3);
            // compute_reward (:189-217): the reference's f64 sum for the step's
            // events, tabulated on the host in its order (TAB_SREW)
            const int gx = goal & 0xff, gy = (goal >> 8) & 0xff, gz = (goal >> 16) & 0xff;
            const bool hit = g.x == gx && g.y == gy && g.z >= gz && g.z - gz < 5;   // SPOT_GOAL_HEIGTH = 5
            if (!moved) g.bumps += 1;
            if (hit) g.done = true;
            const uint32_t ev = (moved ? 0u : 1u) | ((a != 2 && a < 4) ? 2u : 0u) | (hit ? 4u : 0u) |
                                (explored ? 8u : 0u);
            term = g.done;
            const size_t o = (size_t)k * p.N + ai;
            srew[b * 64 + lane] = srt[ev];
            sflg[b * 64 + lane] = (term ? 1u : 0u) | (trunc ? 2u : 0u);
            if (p.reward64) p.reward64[o] = srt64[ev];
            if ((term || trunc) && p.autoreset && p.terminal_obs) {
                float *to = p.terminal_obs + o * OD;
                for (int q = 0; q < OD; ++q) to[q] = row[q];
            }
        }
        SB_T(4);
        // SB3 VecEnv auto-reset
        const bool need = live && p.autoreset && (term || trunc) && !(VN_ABLATE & 512u);
        if (__ballot(need)) {
            sl_reset_wave<LMAX>(p, pl, need, live, next_seed, g, goal, R, w, row, lane, a0, nd, mt_lds, lx, ly);
            if (need) {
                next_seed += p.seed_stride;
                dirty = 3u;                              // the start cell's lines (LDS only)
            }
            // from the start cell (the wave's loads are issued together)
            premove(k + 1, need && k + 1 < p.K, true);
        }
        SB_T(5);
        lds_handoff();                         // hand buffer b to the store wave
        SB_T(6);
    }
#if VN_SIMPLE_PROF
    if (lane == 0) {
        uint64_t tot = 0;
        for (int q = 0; q < 7; ++q) {
            atomicAdd(&g_simple_prof[q], (unsigned long long)prof[q]);
            tot += prof[q];
        }
        atomicAdd(&g_simple_prof[7], tot);
        atomicAdd(&g_simple_prof[8], 1ull);
    }
#endif
    sl_pair_store(brs, (live && (dirty & 1u)) ? xline_off(g.y) : SL_OFF, sl_lds_get(lx), odd);
    sl_pair_store(brs, (live && (dirty & 2u)) ? yline_off(g.x) : SL_OFF, sl_lds_get(ly), odd);
    if (live) {
        p.hot[ai] = pack(g);
        p.goal[ai] = goal;
        p.next_seed[ai] = next_seed;
        p.predraw[ai] = nd;
    }
    (void)L;
}

// internal_grid value of one cell from S, Q and the walls (see the layout
// note above the bit-plane kernel)
__device__ int8_t sb_belief_cell(const Params &p, int i, const Room &R, int x, int y, int z) {
    const SPlanes pl = splanes(p, i);
    auto wall = [&](int cx, int cy, int cz) {
        return ((p.rays[R.ray_off + (uint32_t)((cx * R.D + cy) * R.H + cz)].y >> 16) & 1u) != 0u;
    };
    auto sbit = [&](int cx, int cy, int cz) {
        if (p.sline) return ((reinterpret_cast<const uint32_t *>(pl.sx)[cy * p.ph + cz] >> cx) & 1u) != 0u;
        return ((pl.sz[cx * p.pd + cy] >> cz) & 1u) != 0u;
    };
    const bool is_wall = wall(x, y, z);
    if (!is_wall && ((pl.qz[x * p.pd + y] >> z) & 1u)) return 2;
    if (sbit(x, y, z)) return 1;
    static constexpr int DX[6] = {1, -1, 0, 0, 0, 0}, DY[6] = {0, 0, 1, -1, 0, 0}, DZ[6] = {0, 0, 0, 0, 1, -1};
    for (int d = 0; d < 6; ++d) {
        for (int s = 1; s <= p.L; ++s) {   // a sensing position p = c - s * d, free cells in between
            const int px = x - DX[d] * s, py = y - DY[d] * s, pz = z - DZ[d] * s;
            if (px < 0 || px >= R.W || py < 0 || py >= R.D || pz < 0 || pz >= R.H || wall(px, py, pz)) break;
            if (sbit(px, py, pz)) return is_wall ? 2 : 0;
        }
    }
    return -1;
}

__global__ void export_belief_simple_kernel(Params p, int8_t *out, int pw, int pd) {
    const size_t cells = (size_t)pw * pd * p.ph;
    const size_t gid = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (gid >= cells * (size_t)p.N) return;
    const int i = (int)(gid / cells);
    const size_t c = gid - (size_t)i * cells;
    const int z = (int)(c % p.ph), y = (int)((c / p.ph) % pd), x = (int)(c / ((size_t)p.ph * pd));
    const Agent g = unpack(p.hot[i]);
    const Room R = load_room(p, g.room);
    int8_t v = -128;
    if (x < R.W && y < R.D && z < R.H && p.sbits)
        v = sb_belief_cell(p, i, R, x, y, z);
    else if (x < R.W && y < R.D && z < R.H)
        v = p.belief[(size_t)i * p.agent_bytes + (size_t)(x * p.pd + y) * p.ph + z];
    out[gid] = v;
}

}  // namespace

namespace vn_simple {

// Params crosses the unit boundary as a pointer: each unit has its own
// (identical) copy of the anonymous-namespace layout from env_core.h.

int ensure_mt(int device) { return ensure_mt_table(device); }

// The simpleEnv kernel for a call shape: the line layout's step kernel
// (rooms <= 32 x 32 x 8), the word layout's (<= 64 x 64 x 31), the bit-plane
// reset kernel for both, the dense-map kernel for larger rooms.
template <int LM>
static int launch_lm(bool reset_only, int sline, int sbits, int N, int obs_dim, const Params &p, hipStream_t s) {
    if (!reset_only && sline) {
        // stepping wave + store wave per 64 agents (simple_line_kernel)
        const size_t lds = (size_t)2 * 64 * obs_dim * sizeof(float) + 2 * 64 * 8 + 64 * MT_WS * 4 +
                           (4 + 3 * 64 * SL_STRIDE) * 4 + SL_CLUT * 16 + 48 * 4;
        const dim3 grid((unsigned)((N + 63) / 64));
        if (p.actions) hipLaunchKernelGGL((simple_line_kernel<LM, true>), grid, dim3(128), lds, s, p);
        else hipLaunchKernelGGL((simple_line_kernel<LM, false>), grid, dim3(128), lds, s, p);
    } else if (!reset_only && sbits) {
        // software-pipelined stepping wave + store wave per 64 agents (simple_pipe_kernel)
        const size_t lds = (size_t)2 * 64 * obs_dim * sizeof(float) + 2 * 64 * 8 + 64 * MT_WS * 4;
        const dim3 grid((unsigned)((N + 63) / 64));
        if (p.actions) hipLaunchKernelGGL((simple_pipe_kernel<LM, true>), grid, dim3(128), lds, s, p);
        else hipLaunchKernelGGL((simple_pipe_kernel<LM, false>), grid, dim3(128), lds, s, p);
    } else if (sbits) {
        const size_t lds = (size_t)64 * obs_dim * sizeof(float);
        hipLaunchKernelGGL((simple_bits_reset_kernel<LM>), dim3((unsigned)((N + 63) / 64)), dim3(64), lds, s, p);
    } else {
        const size_t lds = (size_t)64 * obs_dim * sizeof(float);
        const dim3 grid((unsigned)((N + 63) / 64));
        if (reset_only) hipLaunchKernelGGL((simple_kernel<true>), grid, dim3(64), lds, s, p);
        else hipLaunchKernelGGL((simple_kernel<false>), grid, dim3(64), lds, s, p);
    }
    VN_HIP(hipGetLastError());
    return VN_OK;
}

int launch(bool reset_only, int sline, int sbits, int L, int N, int obs_dim, const void *params, hipStream_t s) {
    const Params &p = *static_cast<const Params *>(params);
    if (L <= 4) return launch_lm<4>(reset_only, sline, sbits, N, obs_dim, p, s);
    if (L <= 8) return launch_lm<8>(reset_only, sline, sbits, N, obs_dim, p, s);
    if (L <= 10) return launch_lm<10>(reset_only, sline, sbits, N, obs_dim, p, s);
    return launch_lm<16>(reset_only, sline, sbits, N, obs_dim, p, s);
}

std::string label(bool reset_only, bool ext, int sline, int sbits, int L) {
    char buf[96];
    const int lmax = L <= 4 ? 4 : L <= 8 ? 8 : L <= 10 ? 10 : 16;
    if (!reset_only && sline)
        std::snprintf(buf, sizeof(buf), "simple_line_kernel<%d, %s>", lmax, ext ? "true" : "false");
    else if (!reset_only && sbits)
        std::snprintf(buf, sizeof(buf), "simple_pipe_kernel<%d, %s>", lmax, ext ? "true" : "false");
    else if (sbits)
        std::snprintf(buf, sizeof(buf), "simple_bits_reset_kernel<%d>", lmax);
    else
        std::snprintf(buf, sizeof(buf), "simple_kernel<%s>", reset_only ? "true" : "false");
    return buf;
}

int export_belief(const void *params, int8_t *out, int pw, int pd, hipStream_t s) {
    const Params &p = *static_cast<const Params *>(params);
    const size_t total = (size_t)p.N * pw * pd * p.ph;
    hipLaunchKernelGGL(export_belief_simple_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, p, out,
                       pw, pd);
    VN_HIP(hipGetLastError());
    return VN_OK;
}

}  // namespace vn_simple

#if VN_SIMPLE_PROF
extern "C" int vn_debug_simple_prof(unsigned long long *out16, int clear) {
    VN_HIP(hipMemcpyFromSymbol(out16, HIP_SYMBOL(g_simple_prof), sizeof(unsigned long long) * 16));
    if (clear) {
        unsigned long long z[16] = {0};
        VN_HIP(hipMemcpyToSymbol(HIP_SYMBOL(g_simple_prof), z, sizeof(z)));
    }
    return VN_OK;
}
#endif
