// What bounds the traversal loop: a dependent random gather per lane (each
// step's address comes from the previous step's data, like a BVH descent),
// with the load shapes of the pool kernels, on tables that live in L2
// (2 MiB), in the Infinity Cache (64 MiB) or in HBM (2 GiB).
//
//   P1   one 16-B load per lane per step
//   P3   three 16-B loads of one 48-B slot (a primitive test)
//   P4   four 16-B loads of one 64-B node (a quantized-node step)
//   P7   a 64-B node and a 48-B slot from two independent chains (the
//        overlapped node + primitive step of trace_spec)
//   C4   the 64-B node step loaded cooperatively: each instruction, four
//        neighbouring lanes read the four quarters of one lane's node (16
//        nodes, 16 lines per instruction instead of 64), handed to the
//        owning lane through LDS (4 ds_write_b128 + 4 ds_read_b128)
//
// Prints steps/s, lane-loads per clock per CU and the time of a step per
// wave, for 2..8 waves per SIMD.  hipcc --offload-arch=gfx950 -O3
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                                 \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                           \
        }                                                                                      \
    } while (0)

__device__ __forceinline__ uint32_t hash(uint32_t v) {
    uint32_t s = v * 747796405u + 2891336453u;
    uint32_t w = ((s >> ((s >> 28u) + 4u)) ^ s) * 277803737u;
    return (w >> 22u) ^ w;
}

// table of 64-B granules; word 0 of every 16-B quarter holds a random granule index
__global__ void k_init(uint4* t, uint32_t granules) {
    for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < granules * 4u; i += gridDim.x * blockDim.x)
        t[i] = make_uint4(hash(i) % granules, hash(i ^ 0x55u), hash(i ^ 0xAAu), hash(i ^ 0xFFu));
}

template <int P>
__global__ __launch_bounds__(256) void k_chase(const uint4* __restrict__ t, uint32_t granules, uint32_t steps,
                                              uint32_t* sink) {
    __shared__ uint4 xfer[256 * 4];
    const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t a = hash(gid) % granules, b = hash(gid ^ 0x1234567u) % granules;
    uint32_t acc = 0;
    for (uint32_t s = 0; s < steps; s++) {
        if constexpr (P == 1) {
            const uint4 q = t[4 * a];
            a = q.x;
            acc ^= q.y;
        } else if constexpr (P == 3) {
            const uint4* g = t + 4 * a;
            const uint4 q0 = g[0], q1 = g[1], q2 = g[2];
            a = (q0.x ^ q1.y ^ q2.z) % granules;
            acc ^= q1.x;
        } else if constexpr (P == 4) {
            const uint4* g = t + 4 * a;
            const uint4 q0 = g[0], q1 = g[1], q2 = g[2], q3 = g[3];
            a = (q0.x ^ q1.y ^ q2.z ^ q3.w) % granules;
            acc ^= q3.x;
        } else if constexpr (P == 7) {
            const uint4* g = t + 4 * a;
            const uint4* h = t + 4 * b;
            const uint4 q0 = g[0], q1 = g[1], q2 = g[2], q3 = g[3];
            const uint4 r0 = h[0], r1 = h[1], r2 = h[2];
            a = (q0.x ^ q1.y ^ q2.z ^ q3.w) % granules;
            b = (r0.x ^ r1.y ^ r2.z) % granules;
            acc ^= q3.x ^ r2.x;
        } else if constexpr (P >= 100) {  // P4 with only (P - 100)% of the lanes stepping
            // 1xx: the idle lanes are masked off (exec); 2xx: they load granule 0
            // (what the traversal's unconditional loads do)
            const uint32_t pct = P % 100;
            const bool on = (hash(gid * 31u + s) % 100u) < pct;
            if constexpr (P >= 300) {  // 3xx: buffer loads, idle lanes out of the buffer's range (no fetch)
                const __amdgpu_buffer_rsrc_t rs =
                    __builtin_amdgcn_make_buffer_rsrc(const_cast<uint4*>(t), (short)0, (int)(granules * 64u), 0x00020000);
                const uint32_t off = on ? a * 64u : 0xFFFFFF00u;  // (+48 must not wrap into range)
                const uint4 q0 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
                const uint4 q1 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 16u, 0, 0));
                const uint4 q2 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 32u, 0, 0));
                const uint4 q3 = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off + 48u, 0, 0));
                const uint32_t na = (q0.x ^ q1.y ^ q2.z ^ q3.w) % granules;
                a = on ? na : a;
                acc ^= on ? q3.x : 0u;
            } else if constexpr (P < 200) {
                if (on) {
                    const uint4* g = t + 4 * a;
                    const uint4 q0 = g[0], q1 = g[1], q2 = g[2], q3 = g[3];
                    a = (q0.x ^ q1.y ^ q2.z ^ q3.w) % granules;
                    acc ^= q3.x;
                }
            } else {
                const uint4* g = t + 4 * (on ? a : 0u);
                const uint4 q0 = g[0], q1 = g[1], q2 = g[2], q3 = g[3];
                const uint32_t na = (q0.x ^ q1.y ^ q2.z ^ q3.w) % granules;
                a = on ? na : a;
                acc ^= on ? q3.x : 0u;
            }
        } else {  // C4: cooperative node loads
            const uint32_t lane = __lane_id(), wbase = threadIdx.x & ~63u;
            uint4 v[4];
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint32_t owner = k * 16 + (lane >> 2);
                const uint32_t ai = __shfl(a, owner);
                v[k] = t[4 * ai + (lane & 3u)];
            }
#pragma unroll
            for (int k = 0; k < 4; k++) xfer[(wbase + k * 16 + (lane >> 2)) * 4 + (lane & 3u)] = v[k];
            __builtin_amdgcn_wave_barrier();
            const uint4 q0 = xfer[threadIdx.x * 4], q1 = xfer[threadIdx.x * 4 + 1], q2 = xfer[threadIdx.x * 4 + 2],
                        q3 = xfer[threadIdx.x * 4 + 3];
            __builtin_amdgcn_wave_barrier();
            a = (q0.x ^ q1.y ^ q2.z ^ q3.w) % granules;
            acc ^= q3.x;
        }
    }
    if (acc == 0x12345678u && a == 7u) sink[0] = acc;
}

template <int P>
static void run(const uint4* t, uint32_t granules, int cus, int waves_per_simd, uint32_t steps, uint32_t* sink,
                double clock_ghz, const char* tname) {
    // 256-thread blocks = 4 waves; waves_per_simd blocks per CU
    const int blocks = cus * waves_per_simd;
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    hipLaunchKernelGGL(k_chase<P>, dim3(blocks), dim3(256), 0, 0, t, granules, steps / 8, sink);  // warm
    CHK(hipEventRecord(e0));
    hipLaunchKernelGGL(k_chase<P>, dim3(blocks), dim3(256), 0, 0, t, granules, steps, sink);
    CHK(hipEventRecord(e1));
    CHK(hipEventSynchronize(e1));
    float ms = 0;
    CHK(hipEventElapsedTime(&ms, e0, e1));
    const int loads = P == 1 ? 1 : P == 3 ? 3 : P == 4 ? 4 : P == 7 ? 7 : 4;  // lane-loads counted for every lane
    const double wave_steps = (double)blocks * 4 * steps;
    const double lane_loads = wave_steps * 64 * loads;
    const double cycles = ms * 1e-3 * clock_ghz * 1e9;
    printf("%-6s P%-2d waves/SIMD %d  %8.2f ms  %7.2f G wave-steps/s  %6.3f lane-loads/clk/CU  %7.0f clk/step/wave\n",
           tname, P, waves_per_simd, ms, wave_steps / (ms * 1e-3) / 1e9, lane_loads / cycles / cus,
           cycles / (wave_steps / (blocks * 4.0)));
    CHK(hipEventDestroy(e0));
    CHK(hipEventDestroy(e1));
}

int main(int argc, char** argv) {
    hipDeviceProp_t p;
    CHK(hipGetDeviceProperties(&p, 0));
    const int cus = p.multiProcessorCount;
    const double ghz = argc > 1 ? atof(argv[1]) : 2.4;
    printf("%s, %d CUs, clock taken as %.2f GHz\n", p.name, cus, ghz);
    uint32_t* sink;
    CHK(hipMalloc(&sink, 64));
    const struct { const char* name; size_t bytes; uint32_t steps; } tabs[] = {
        {"L2", 2ull << 20, 4096}, {"MALL", 64ull << 20, 2048}, {"HBM", 2ull << 30, 1024}};
    if (argc > 2 && atoi(argv[2]) == 1) {  // masked vs dummy loads at 30 / 70 / 100 % active lanes
        const uint32_t granules = (uint32_t)((2ull << 20) / 64);
        uint4* t;
        CHK(hipMalloc(&t, 2ull << 20));
        hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, t, granules);
        CHK(hipDeviceSynchronize());
        for (int w : {4, 6}) {
            run<130>(t, granules, cus, w, 4096, sink, ghz, "L2m30");
            run<230>(t, granules, cus, w, 4096, sink, ghz, "L2d30");
            run<170>(t, granules, cus, w, 4096, sink, ghz, "L2m70");
            run<270>(t, granules, cus, w, 4096, sink, ghz, "L2d70");
            run<330>(t, granules, cus, w, 4096, sink, ghz, "L2b30");
            run<370>(t, granules, cus, w, 4096, sink, ghz, "L2b70");
            run<4>(t, granules, cus, w, 4096, sink, ghz, "L2all");
        }
        CHK(hipFree(t));
        return 0;
    }
    for (const auto& tb : tabs) {
        const uint32_t granules = (uint32_t)(tb.bytes / 64);
        uint4* t;
        CHK(hipMalloc(&t, tb.bytes));
        hipLaunchKernelGGL(k_init, dim3(4096), dim3(256), 0, 0, t, granules);
        CHK(hipDeviceSynchronize());
        for (int w : {2, 4, 6, 8}) {
            run<1>(t, granules, cus, w, tb.steps, sink, ghz, tb.name);
            run<3>(t, granules, cus, w, tb.steps, sink, ghz, tb.name);
            run<4>(t, granules, cus, w, tb.steps, sink, ghz, tb.name);
            run<7>(t, granules, cus, w, tb.steps, sink, ghz, tb.name);
            run<5>(t, granules, cus, w, tb.steps, sink, ghz, tb.name);  // C4
        }
        CHK(hipFree(t));
    }
    CHK(hipFree(sink));
    return 0;
}
