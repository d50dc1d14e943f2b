// Does a wave's vector-memory load cost per instruction or per byte?  (round 6, C4: the global-scene
// kernel's TA / TD are 0.93 / 0.98 busy and 87 % of its vector loads are the four dwordx4 reads of a
// 64-B quantised node; a smaller node pays only if the cost follows bytes.)
//
// Every lane of a persistent grid (256-thread blocks, 6 waves per SIMD as the global-scene kernel)
// runs a dependent chain of node reads from a node array of `kib` KiB (64-B nodes, distinct per lane).
// Per node it issues `n` loads of `w` bytes each (w = 4, 8, 12, 16) at offsets 0, 16, 32, 48 of the
// node.  Kernel time per wave-instruction, against (w, n), separates the per-instruction from the
// per-byte cost.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/l1_width tools/micro/l1_width.hip && /tmp/l1_width [KiB]
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

constexpr int kIters = 2048;

// quad-cooperative read: the four lanes of a quad read the four 16-B chunks of ONE node (one dwordx4
// instruction per node and quad; MODE 0), or all four lanes read the same chunk (MODE 1, the
// uniform-quad case of l1_lines.hip), or each lane its own node's chunk (MODE 2, scattered)
template <int MODE>
__global__ __launch_bounds__(256) void chase_quad(const uint32_t* __restrict__ nodes, uint32_t n_nodes, uint32_t seed,
                                                  float* out) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t q = MODE == 2 ? tid : tid >> 2, j = tid & 3u;
    uint32_t h = (q * 0x9E3779B9u) ^ seed;
    uint32_t acc = 0;
    for (int i = 0; i < kIters; ++i) {
        h = h * 747796405u + 2891336453u;
        const uint32_t idx = (h >> 8) % n_nodes;
        const uint32_t* p = nodes + (size_t)idx * 16 + (MODE == 1 ? 0u : 4u * j);
        const uint4 v = *reinterpret_cast<const uint4*>(p);
        acc += v.x ^ v.y ^ v.z ^ v.w;
        h ^= acc & 1u;
    }
    if (acc == 0x12345u) out[0] = (float)acc;
}

template <int MODE>
void run_quad(const uint32_t* d_nodes, uint32_t n_nodes, int grid, float* d_out, int cus, bool& first) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    chase_quad<MODE><<<grid, 256>>>(d_nodes, n_nodes, 1u, d_out);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) chase_quad<MODE><<<grid, 256>>>(d_nodes, n_nodes, 2u + r, d_out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0.0f;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double wave_insts = 3.0 * grid * 4 * kIters;
    static const char* names[3] = {"quad reads one node's four chunks", "quad reads one chunk", "lanes read own nodes"};
    std::printf("%s {\"quad_mode\": \"%s\", \"ms\": %.3f, \"ns_per_wave_inst_per_cu\": %.3f}", first ? "" : ",\n",
                names[MODE], ms / 3.0, ms * 1e6 / wave_insts * cus);
    first = false;
}

template <int W, int N>
__global__ __launch_bounds__(256) void chase(const uint32_t* __restrict__ nodes, uint32_t n_nodes, uint32_t seed,
                                             float* out) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    uint32_t h = (tid * 0x9E3779B9u) ^ seed;
    uint32_t acc = 0;
    for (int i = 0; i < kIters; ++i) {
        h = h * 747796405u + 2891336453u;
        const uint32_t idx = (h >> 8) % n_nodes;
        const uint32_t* nd = nodes + (size_t)idx * 16;
#pragma unroll
        for (int k = 0; k < N; ++k) {
            const uint32_t* p = nd + 4 * k;
            if constexpr (W == 16) {
                const uint4 v = *reinterpret_cast<const uint4*>(p);
                acc += v.x ^ v.y ^ v.z ^ v.w;
            } else if constexpr (W == 12) {
                const uint3 v = *reinterpret_cast<const uint3*>(p);
                acc += v.x ^ v.y ^ v.z;
            } else if constexpr (W == 8) {
                const uint2 v = *reinterpret_cast<const uint2*>(p);
                acc += v.x ^ v.y;
            } else {
                acc += *p;
            }
        }
        // the next index waits for this node (a traversal's dependent chain)
        h ^= acc & 1u;
    }
    if (acc == 0x12345u) out[0] = (float)acc;
}

template <int W, int N>
void run(const uint32_t* d_nodes, uint32_t n_nodes, int grid, float* d_out, int cus, bool& first) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    chase<W, N><<<grid, 256>>>(d_nodes, n_nodes, 1u, d_out);   // warm
    hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) chase<W, N><<<grid, 256>>>(d_nodes, n_nodes, 2u + r, d_out);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0.0f;
    hipEventElapsedTime(&ms, e0, e1);
    const double wave_insts = 3.0 * grid * 4 * kIters * N;
    std::printf("%s {\"bytes\": %d, \"loads_per_node\": %d, \"ms\": %.3f, \"ns_per_wave_inst_per_cu\": %.3f, "
                "\"ns_per_node_per_cu\": %.3f}",
                first ? "" : ",\n", W, N, ms / 3.0, ms * 1e6 / wave_insts * cus, ms * 1e6 / wave_insts * N * cus);
    first = false;
    hipEventDestroy(e0);
    hipEventDestroy(e1);
}

int main(int argc, char** argv) {
    const uint32_t kib = argc > 1 ? (uint32_t)atoi(argv[1]) : 2u << 10;
    const uint32_t n_nodes = kib << 10 >> 6;
    std::vector<uint32_t> host((size_t)n_nodes * 16);
    for (size_t i = 0; i < host.size(); ++i) host[i] = (uint32_t)(i * 2654435761u);
    uint32_t* d_nodes;
    float* d_out;
    hipMalloc(&d_nodes, host.size() * 4);
    hipMalloc(&d_out, 4);
    hipMemcpy(d_nodes, host.data(), host.size() * 4, hipMemcpyHostToDevice);
    hipDeviceProp_t prop;
    hipGetDeviceProperties(&prop, 0);
    const int grid = prop.multiProcessorCount * 6;
    std::printf("{\"cus\": %d, \"iters\": %d, \"kib\": %u, \"rows\": [\n", prop.multiProcessorCount, kIters, kib);
    bool first = true;
    run<16, 4>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    run<16, 3>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    run<16, 2>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    run<16, 1>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    run<12, 4>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    run<8, 4>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    run<4, 4>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    run_quad<0>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    run_quad<1>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    run_quad<2>(d_nodes, n_nodes, grid, d_out, prop.multiProcessorCount, first);
    std::printf("\n]}\n");
    hipFree(d_nodes);
    hipFree(d_out);
    return 0;
}
