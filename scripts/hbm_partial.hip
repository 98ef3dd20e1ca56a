// hbm_partial.hip -- what scattered small stores cost beside the env step's
// obs stream.  The env kernels' geometry: 65,536 agents x 4
// lanes, K steps per launch, per agent-step the 80-float obs row (a wave's 16
// rows as five 1-KiB non-temporal stores) plus `n` extra stores into the
// agent's own 32 KiB region (a PH-16 belief map) at pseudo-random offsets:
//   mode 0  obs only (n ignored)
//   mode 1  n 1-B stores, one lane each (a blind byte mark)
//   mode 2  n 8-B stores, one lane each (a plane-row word)
//   mode 3  n 8-B read-modify-writes, one lane each (load the word, store it back
//           changed: the plane row the step loaded, then marked)
//   mode 4  n 64-B stores, 16 B per lane of the agent's 4 (a whole piece)
//   mode 5  n 16-B stores, one lane each (a window column written back)
//   mode 6  n 64-B pieces, each written by ONE lane as four 16-B stores (a
//           padded column: does L2 merge them into one whole-piece write-back?)
//   mode 7  n 32-B half pieces, one lane, two 16-B stores
// A diagnostic, not product.
//
//   hipcc -O3 --offload-arch=gfx950 scripts/hbm_partial.hip -o scripts/hbm_partial
//   scripts/hbm_partial [K=128] [launches=10] [first mode=0]
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

constexpr int REGION = 32768, OBS = 80;

__device__ __forceinline__ uint32_t mix(uint32_t a, uint32_t b) {
    uint32_t h = a * 2654435761u ^ b * 40503u;
    h ^= h >> 13;
    h *= 0x5bd1e995u;
    return h ^ (h >> 15);
}

__global__ __launch_bounds__(256) void partial_kernel(uint8_t *__restrict__ region, float *__restrict__ obs, int N,
                                                      int K, int mode, int n, uint32_t salt,
                                                      uint32_t *__restrict__ sink) {
    const int lane = threadIdx.x & 63, q = threadIdx.x & 3;
    const int agent = (int)((blockIdx.x * blockDim.x + threadIdx.x) >> 2);
    const int wave_agent0 = (int)((blockIdx.x * blockDim.x + (threadIdx.x & ~63)) >> 2);
    uint8_t *r = region + (size_t)agent * REGION;
    uint32_t acc = salt;
    for (int k = 0; k < K; ++k) {
        for (int pc = 0; pc < n && mode != 0; ++pc) {
            const uint32_t h = mix((uint32_t)agent, (uint32_t)(k * 16 + pc) ^ salt);
            const int owner = pc & 3;
            if (mode == 1) {
                if (q == owner) r[h & (REGION - 1)] = (uint8_t)acc;
            } else if (mode == 2) {
                if (q == owner) reinterpret_cast<uint64_t *>(r)[h & (REGION / 8 - 1)] = acc;
            } else if (mode == 3) {
                if (q == owner) {
                    uint64_t *w = reinterpret_cast<uint64_t *>(r) + (h & (REGION / 8 - 1));
                    const uint64_t v = *w;
                    *w = v | (1ull << (acc & 63));
                }
            } else if (mode == 4) {
                reinterpret_cast<uint4 *>(r)[(h & (REGION / 64 - 1)) * 4 + q] = make_uint4(acc, acc, acc, acc);
            } else if (mode == 5) {
                if (q == owner) reinterpret_cast<uint4 *>(r)[h & (REGION / 16 - 1)] = make_uint4(acc, acc, acc, acc);
            } else {
                if (q == owner) {
                    uint4 *w = reinterpret_cast<uint4 *>(r) + (h & (REGION / 64 - 1)) * 4;
#pragma unroll
                    for (int j = 0; j < (mode == 6 ? 4 : 2); ++j) w[j] = make_uint4(acc, acc, j, 0u);
                }
            }
        }
        F4v *dst = reinterpret_cast<F4v *>(obs + ((size_t)k * N + wave_agent0) * OBS);
        const float x = (float)(acc & 0xff);
#pragma unroll
        for (int jj = 0; jj < 5; ++jj) __builtin_nontemporal_store(F4v{x, x, x, x}, dst + lane + 64 * jj);
        acc = acc * 1664525u + 1013904223u;
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char **argv) {
    const int N = 65536, K = argc > 1 ? std::atoi(argv[1]) : 128, L = argc > 2 ? std::atoi(argv[2]) : 10;
    uint8_t *region;
    float *obs;
    uint32_t *sink;
    CK(hipMalloc(&region, (size_t)N * REGION));
    CK(hipMalloc(&obs, (size_t)K * N * OBS * sizeof(float)));
    CK(hipMalloc(&sink, 4));
    CK(hipMemset(region, 0, (size_t)N * REGION));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const char *names[8] = {"obs only", "1-B stores", "8-B stores", "8-B read-modify-writes", "64-B stores (4 lanes)",
                            "16-B stores", "64-B pieces, one lane, 4 x 16 B", "32-B half pieces, one lane, 2 x 16 B"};
    const int m0 = argc > 3 ? std::atoi(argv[3]) : 0;
    const int ns[4] = {1, 2, 3, 4};
    for (int mode = m0; mode < 8; ++mode) {
        for (int ni = 0; ni < (mode == 0 ? 1 : 4); ++ni) {
            const int n = mode == 0 ? 0 : ns[ni];
            for (int w = 0; w < 2; ++w)
                hipLaunchKernelGGL(partial_kernel, dim3(N * 4 / 256), dim3(256), 0, 0, region, obs, N, K, mode, n, 7u,
                                   sink);
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0));
            for (int l = 0; l < L; ++l)
                hipLaunchKernelGGL(partial_kernel, dim3(N * 4 / 256), dim3(256), 0, 0, region, obs, N, K, mode, n,
                                   (uint32_t)l * 977u, sink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms = 0.f;
            CK(hipEventElapsedTime(&ms, e0, e1));
            const double us = ms * 1e3 / L, steps = (double)N * K;
            std::printf("{\"mode\": \"%s\", \"n_per_agent_step\": %d, \"K\": %d, \"us_per_launch\": %.1f, "
                        "\"ns_per_step\": %.1f, \"G_agent_steps_per_s\": %.3f}\n",
                        names[mode], n, K, us, us * 1e3 / K, steps / us * 1e-3);
            std::fflush(stdout);
        }
    }
    return 0;
}
