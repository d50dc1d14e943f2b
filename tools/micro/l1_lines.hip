// Does the vector-L1 pipeline cost of a wave's node load depend on how many DISTINCT lines its lanes
// touch?  (round 6, VERDICT r05 item 6: tools/coherence_c4.cpp prices an origin-sorted ray stage at
// -17 % distinct lines per node load at config 4; the sort pays only if the kernel's TA / TD-bound
// loads get cheaper with fewer distinct lines, not only with fewer lanes or bytes.)
//
// Every lane of a persistent grid (256-thread blocks, 6 waves per SIMD as the global-scene kernel)
// runs a dependent chain of 64-B node loads (four dwordx4, the quantised BVH4 node) from an 11 MB array
// (config 4's quantised nodes); the next index depends on the loaded data, as in a traversal.  Lanes
// share a node in groups of `share` (1: 64 distinct lines per load, 64: one line); `active` lanes of
// each wave load (the others idle, as divergent traversal lanes).  Kernel time per wave-load over the
// sharing factors tells whether distinct lines, not lanes, set the cost.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/l1_lines tools/micro/l1_lines.hip && /tmp/l1_lines [KiB]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kIters = 2048;

__global__ __launch_bounds__(256) void chase(const float4* __restrict__ nodes, uint32_t n_nodes, int share, int active,
                                             uint32_t seed, float* out) {
    const int lane = threadIdx.x & 63;
    const uint32_t wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (lane >= active) return;
    const uint32_t group = (uint32_t)(lane / share);
    uint32_t h = (wave * 0x9E3779B9u) ^ (group * 0x85EBCA6Bu) ^ seed;
    float acc = 0.0f;
    for (int i = 0; i < kIters; ++i) {
        h = h * 747796405u + 2891336453u;
        const uint32_t idx = (h >> 8) % n_nodes;
        const float4* nd = nodes + (size_t)idx * 4;
        const float4 a = nd[0], b = nd[1], c = nd[2], d = nd[3];
        acc += a.x + b.y + c.z + d.w;
        // the next index waits for this load (a traversal's dependent chain)
        h ^= __float_as_uint(acc) & 1u;
    }
    if (acc == 12345.0f) out[0] = acc;
}

int main(int argc, char** argv) {
    // node array size in KiB (default 11 MiB, config 4's quantised nodes; 16 KiB stays in the vector L1,
    // 2 MiB in L2)
    const uint32_t kib = argc > 1 ? (uint32_t)atoi(argv[1]) : 11u << 10;
    const uint32_t n_nodes = kib << 10 >> 6;
    std::vector<float> host((size_t)n_nodes * 16);
    for (size_t i = 0; i < host.size(); ++i) host[i] = (float)(i % 7) * 1e-3f;
    float4* d_nodes;
    float* d_out;
    hipMalloc(&d_nodes, host.size() * 4);
    hipMalloc(&d_out, 4);
    hipMemcpy(d_nodes, host.data(), host.size() * 4, hipMemcpyHostToDevice);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int grid = prop.multiProcessorCount * 6;   // 6 blocks of 4 waves per CU = 6 waves per SIMD
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    std::printf("{\"cus\": %d, \"iters\": %d, \"kib\": %u, \"rows\": [\n", prop.multiProcessorCount, kIters, kib);
    bool first = true;
    for (int active : {64, 32}) {
        for (int share : {1, 2, 4, 8, 16, 64}) {
            chase<<<grid, 256>>>(d_nodes, n_nodes, share, active, 1u, d_out);   // warm
            hipEventRecord(e0);
            for (int r = 0; r < 3; ++r) chase<<<grid, 256>>>(d_nodes, n_nodes, share, active, 2u + r, d_out);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms = 0.0f;
            hipEventElapsedTime(&ms, e0, e1);
            const double wave_loads = 3.0 * grid * 4 * kIters;   // per 64-B node load (4 instructions)
            std::printf("%s {\"active\": %d, \"share\": %d, \"distinct_lines\": %d, \"ms\": %.3f, \"ns_per_wave_load_per_cu\": %.3f}",
                        first ? "" : ",\n", active, share, (active + share - 1) / share, ms / 3.0,
                        ms * 1e6 / wave_loads * prop.multiProcessorCount);
            first = false;
        }
    }
    std::printf("\n]}\n");
    hipFree(d_nodes);
    hipFree(d_out);
    return 0;
}
