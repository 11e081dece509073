// FETCH_SIZE calibration on the traversal kernels' own access patterns
// (MI355X_MICROARCH.md "HBM": FETCH_SIZE reports half of a wide coalesced
// streaming read on gfx950; other access widths are uncalibrated).
//
// Known byte counts, every line touched exactly once per launch, from a
// 4 GiB table (16x the 256 MiB Infinity Cache, so nothing is re-served
// on-die between launches):
//   k_stream       lane-contiguous 16-B loads                    16 B / lane
//   k_node_gather  one 128-B cluster per lane as 8 x 16-B loads   128 B / lane
//                  (the BVH4 node step of k_closest_pool)
//   k_slot_gather  one 48-B primitive slot per lane, 3 x 16-B    48 B / lane
//                  loads, slots 128-B aligned in pairs of lines  (128-B lines)
//   k_texel_gather two 8-B loads from two random lines per lane   16 B / lane
//                  (k_shade's u8 bilinear texel-pair rows)
// Lanes pick their line through an odd-multiplier bijection of the index, so
// no line repeats and no index array is read.  Nothing is stored unless a
// data-dependent test that never holds passes, so the only traffic is the
// reads.  Run under `rocprofv3 --pmc FETCH_SIZE` and `--kernel-trace
// --stats`; tools/fetch_calib.py turns the per-dispatch counters into
// factors (known bytes / (FETCH_SIZE * 1024)).
//
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o build/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHK(x)                                                                           \
    do {                                                                                 \
        hipError_t e_ = (x);                                                             \
        if (e_ != hipSuccess) {                                                          \
            fprintf(stderr, "%s: %s (%s:%d)\n", #x, hipGetErrorString(e_), __FILE__, __LINE__); \
            exit(1);                                                                     \
        }                                                                                \
    } while (0)

// lines = power of two; odd multiplier => bijection on [0, lines)
__device__ __forceinline__ unsigned long long scatter(unsigned long long i, unsigned long long mask, unsigned mul) {
    return (i * mul + 0x9E3779B9ull) & mask;
}

__global__ void k_fill(float4* t, unsigned long long n) {
    unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    for (; i < n; i += (unsigned long long)gridDim.x * blockDim.x)
        t[i] = make_float4((float)(i & 1023), 1.0f, 2.0f, 3.0f);
}

__global__ void k_stream(const float4* __restrict__ t, unsigned long long n, float* sink) {
    unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 v = t[i];
    float s = v.x + v.y + v.z + v.w;
    if (s == -1.0f) sink[0] = s;
}

__global__ void k_node_gather(const float4* __restrict__ t, unsigned long long n, unsigned long long mask,
                              unsigned mul, float* sink) {
    unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4* q = t + scatter(i, mask, mul) * 8;  // 128-B line
    float4 a = q[0], b = q[1], c = q[2], d = q[3], e = q[4], f = q[5], g = q[6], h = q[7];
    float s = a.x + b.y + c.z + d.w + e.x + f.y + g.z + h.w;
    if (s == -1.0f) sink[0] = s;
}

// the random-line gather ceiling: each lane gathers G independent 128-B lines
// (8G loads in flight per lane) -- what a traversal step could at best move
template <int G>
__global__ void k_node_gather_n(const float4* __restrict__ t, unsigned long long n, unsigned long long mask,
                                unsigned mul, float* sink) {
    unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    float4 v[G][8];
#pragma unroll
    for (int g = 0; g < G; g++) {
        const float4* q = t + scatter(i * G + g, mask, mul) * 8;
#pragma unroll
        for (int k = 0; k < 8; k++) v[g][k] = q[k];
    }
    float s = 0;
#pragma unroll
    for (int g = 0; g < G; g++)
#pragma unroll
        for (int k = 0; k < 8; k++) s += v[g][k].x;
    if (s == -1.0f) sink[0] = s;
}

// one 64-B quantized node per lane (4 x 16-B loads, 64-B aligned): the node
// step of the pool kernels over DevQNode.  Lines chosen as for k_node_gather;
// the node is the line's first or second half by the lane's parity.
__global__ void k_qnode_gather(const float4* __restrict__ t, unsigned long long n, unsigned long long mask,
                               unsigned mul, float* sink) {
    unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4* q = t + scatter(i, mask, mul) * 8 + 4 * (i & 1);
    float4 a = q[0], b = q[1], c = q[2], d = q[3];
    float s = a.x + b.y + c.z + d.w;
    if (s == -1.0f) sink[0] = s;
}

__global__ void k_slot_gather(const float4* __restrict__ t, unsigned long long n, unsigned long long mask,
                              unsigned mul, float* sink) {
    unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const float4* q = t + scatter(i, mask, mul) * 8;  // first 48 B of a 128-B line
    float4 a = q[0], b = q[1], c = q[2];
    float s = a.x + b.y + c.z;
    if (s == -1.0f) sink[0] = s;
}

// k_shade's bilinear lookup into a u8 image (texel_pair_u8): per lane two
// 8-B loads, one from each of two texel rows, i.e. two random lines with 8 of
// their 128 B used (known 16 B per lane; the lines moved are 2 x 128 B)
__global__ void k_texel_gather(const float4* __restrict__ t, unsigned long long n, unsigned long long mask,
                               unsigned mul, float* sink) {
    unsigned long long i = blockIdx.x * (unsigned long long)blockDim.x + threadIdx.x;
    if (i >= n) return;
    const uint2* r0 = reinterpret_cast<const uint2*>(t + scatter(2 * i, mask, mul) * 8) + (i & 15);
    const uint2* r1 = reinterpret_cast<const uint2*>(t + scatter(2 * i + 1, mask, mul) * 8) + (i & 15);
    const uint2 a = *r0, b = *r1;
    if ((a.x ^ a.y ^ b.x ^ b.y) == 0x12345678u) sink[0] = 1.0f;
}

int main(int argc, char** argv) {
    const unsigned long long bytes = 4ull << 30;
    const unsigned long long n16 = bytes / 16, lines = bytes / 128, mask = lines - 1;
    const unsigned long long n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (16ull << 20);  // lanes per gather
    float4* t = nullptr;
    float* sink = nullptr;
    CHK(hipMalloc(&t, bytes));
    CHK(hipMalloc(&sink, 4));
    hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, t, n16);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const unsigned muls[3] = {2654435761u, 40503u * 2u + 1u, 97u};
    for (int rep = 0; rep < 3; rep++) {
        float ms;
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_stream, dim3((unsigned)((n * 8 + 255) / 256)), dim3(256), 0, 0, t, n * 8, sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\":\"k_stream\",\"bytes\":%llu,\"ms\":%.4f}\n", n * 8 * 16, ms);
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_node_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, t, n, mask, muls[rep],
                           sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\":\"k_node_gather\",\"bytes\":%llu,\"ms\":%.4f}\n", n * 128, ms);
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_slot_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, t, n, mask, muls[rep],
                           sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\":\"k_slot_gather\",\"bytes\":%llu,\"ms\":%.4f}\n", n * 48, ms);
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_qnode_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, t, n, mask, muls[rep],
                           sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\":\"k_qnode_gather\",\"bytes\":%llu,\"ms\":%.4f}\n", n * 64, ms);
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_texel_gather, dim3((unsigned)((n / 2 + 255) / 256)), dim3(256), 0, 0, t, n / 2, mask,
                           muls[rep], sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\":\"k_texel_gather\",\"bytes\":%llu,\"ms\":%.4f,\"lines\":%llu}\n", n / 2 * 16, ms,
               n / 2 * 2);
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_node_gather_n<4>, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, 0, t, n / 4, mask,
                           muls[rep], sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\":\"k_node_gather_n<4>\",\"bytes\":%llu,\"ms\":%.4f}\n", n / 4 * 4 * 128, ms);
        CHK(hipEventRecord(e0));
        hipLaunchKernelGGL(k_node_gather_n<2>, dim3((unsigned)((n / 2 + 255) / 256)), dim3(256), 0, 0, t, n / 2, mask,
                           muls[rep], sink);
        CHK(hipEventRecord(e1));
        CHK(hipEventSynchronize(e1));
        CHK(hipEventElapsedTime(&ms, e0, e1));
        printf("{\"kernel\":\"k_node_gather_n<2>\",\"bytes\":%llu,\"ms\":%.4f}\n", n / 2 * 2 * 128, ms);
    }
    CHK(hipDeviceSynchronize());
    CHK(hipFree(t));
    CHK(hipFree(sink));
    return 0;
}
