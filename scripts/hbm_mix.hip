// hbm_mix.hip -- the env step kernel's memory pattern with no env logic:
// what HBM delivers for the traffic env_kernel<8,false,true,false,2> moves
// (DESIGN.md 7.5).  Per agent and step: two 32-B reads at a pseudo-random
// offset in the agent's own 8 KiB belief region (the entering window column
// and plane set), one 80-float obs row written into [K][N][80] (a wave's 16
// rows are 5 KiB contiguous, 1 KiB per store instruction, non-temporal, as
// the kernel's flush), 4 B reward + 2 B flags.  4 lanes per agent, 65,536
// agents, K steps per launch, 256-thread blocks -- the kernel's geometry.
// Modes: 0 the mix, 1 reads only, 2 writes only.  A diagnostic, not product.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/hbm_mix.hip -o scripts/hbm_mix
//   scripts/hbm_mix [K=64] [launches=20] [read pieces per agent-step=2]
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                                 \
    do {                                                                                      \
        hipError_t e_ = (x);                                                                  \
        if (e_ != hipSuccess) {                                                               \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                      \
            std::exit(1);                                                                     \
        }                                                                                     \
    } while (0)

typedef float F4v __attribute__((ext_vector_type(4)));

constexpr int AGENT_BYTES = 8192, OBS = 80;

__global__ __launch_bounds__(256) void mix_kernel(const uint8_t *__restrict__ belief, float *__restrict__ obs,
                                                  float *__restrict__ rew, uint8_t *__restrict__ flags, int N, int K,
                                                  int mode, int pieces, uint32_t salt, uint32_t *__restrict__ sink) {
    const int lane = threadIdx.x & 63, q = threadIdx.x & 3;
    const int agent = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 2);
    const int wave_agent0 = (int)((blockIdx.x * blockDim.x + (threadIdx.x & ~63)) >> 2);
    uint32_t acc = 0;
    for (int k = 0; k < K; ++k) {
        if (mode != 2) {
            // `pieces` 32-B pieces: lane q reads 8 B of each (one request per agent and piece)
            const uint8_t *b = belief + (size_t)agent * AGENT_BYTES;
            for (int pc = 0; pc < pieces; ++pc) {
                uint32_t h = (uint32_t)agent * 2654435761u ^ (uint32_t)(k * 8 + pc) * 40503u ^ salt;
                h ^= h >> 13;
                const uint32_t o = (h & (AGENT_BYTES / 32 - 1)) * 32;
                const uint2 v = *reinterpret_cast<const uint2 *>(b + o + 8 * q);
                acc += v.x ^ v.y;
            }
        }
        if (mode != 1) {
            // the wave's 16 obs rows: 320 float4, 5 store instructions of 1 KiB
            F4v *dst = reinterpret_cast<F4v *>(obs + ((size_t)k * N + wave_agent0) * OBS);
            const float x = (float)(acc & 0xff);
#pragma unroll
            for (int jj = 0; jj < 5; ++jj) __builtin_nontemporal_store(F4v{x, x, x, x}, dst + lane + 64 * jj);
            if (q == 0) {
                rew[(size_t)k * N + agent] = x;
                flags[2 * ((size_t)k * N + agent)] = (uint8_t)acc;
                flags[2 * ((size_t)k * N + agent) + 1] = (uint8_t)(acc >> 8);
            }
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
    const int N = 65536, K = argc > 1 ? std::atoi(argv[1]) : 64, L = argc > 2 ? std::atoi(argv[2]) : 20;
    const int pieces = argc > 3 ? std::atoi(argv[3]) : 2;
    uint8_t *belief, *flags;
    float *obs, *rew;
    uint32_t *sink;
    CK(hipMalloc(&belief, (size_t)N * AGENT_BYTES));
    CK(hipMalloc(&obs, (size_t)K * N * OBS * sizeof(float)));
    CK(hipMalloc(&rew, (size_t)K * N * sizeof(float)));
    CK(hipMalloc(&flags, (size_t)K * N * 2));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(belief, 1, (size_t)N * AGENT_BYTES));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[3] = {"mix (reads + writes)", "reads only", "writes only"};
    const double rbytes = 32.0 * pieces, wbytes = OBS * 4 + 4 + 2;   // per agent-step
    for (int mode = 0; mode < 3; ++mode) {
        for (int w = 0; w < 3; ++w)
            hipLaunchKernelGGL(mix_kernel, dim3(N * 4 / 256), dim3(256), 0, 0, belief, obs, rew, flags, N, K, mode, pieces,
                               7u, sink);
        CK(hipDeviceSynchronize());
        CK(hipEventRecord(e0));
        for (int l = 0; l < L; ++l)
            hipLaunchKernelGGL(mix_kernel, dim3(N * 4 / 256), dim3(256), 0, 0, belief, obs, rew, flags, N, K, mode,
                               pieces, (uint32_t)l, sink);
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms = 0.f;
        CK(hipEventElapsedTime(&ms, e0, e1));
        const double us = ms * 1e3 / L, steps = (double)N * K;
        const double bytes = steps * ((mode != 2 ? rbytes : 0.0) + (mode != 1 ? wbytes : 0.0));
        std::printf("{\"mode\": \"%s\", \"K\": %d, \"read_pieces\": %d, \"us_per_launch\": %.1f, \"G_agent_steps_per_s\": %.3f, "
                    "\"bytes_per_agent_step\": %.0f, \"TB_per_s\": %.3f}\n",
                    names[mode], K, pieces, us, steps / us * 1e-3, bytes / steps, bytes / us * 1e-6);
    }
    return 0;
}
