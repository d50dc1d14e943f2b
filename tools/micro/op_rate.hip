// Issue-rate probe for a few VALU opcodes on gfx950 (wave64): each thread runs N_ITER rounds of
// 8 independent chains of one operation; kernel time / (waves x ops) gives cycles per wave-op.
//   hipcc --offload-arch=gfx950 -O3 -o /tmp/op_rate tools/micro/op_rate.hip && /tmp/op_rate
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

constexpr int N_ITER = 4096;

template <int OP>
__global__ __launch_bounds__(256) void probe(uint32_t* out, uint32_t seed) {
    uint32_t a[8];
    float f[8];
    for (int k = 0; k < 8; ++k) { a[k] = seed + threadIdx.x * 8 + k; f[k] = (float)a[k] * 1e-3f; }
    for (int i = 0; i < N_ITER; ++i) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            if (OP == 0) f[k] = __builtin_fmaf(f[k], 1.0001f, 0.5f);            // v_fma_f32
            if (OP == 1) a[k] = a[k] * 747796405u;                              // v_mul_lo_u32
            if (OP == 2) a[k] = __umul24(a[k], 0x2a5b3du) + 1u; // v_mad_u32_u24
            if (OP == 3) f[k] = __builtin_amdgcn_rcpf(f[k]);                    // v_rcp_f32
            if (OP == 4) f[k] = __builtin_amdgcn_sqrtf(f[k] + 1.0f);            // v_add + v_sqrt_f32
            if (OP == 5) { uint64_t m = (uint64_t)a[k] * 2891336453ull + a[k]; a[k] = (uint32_t)(m >> 7); } // v_mad_u64_u32
            // opaque to the optimiser: no strength reduction of the chains, no packed (SLP) forms
            asm volatile("" : "+v"(a[k]), "+v"(f[k]));
        }
    }
    uint32_t r = 0;
    for (int k = 0; k < 8; ++k) r ^= a[k] ^ __float_as_uint(f[k]);
    out[blockIdx.x * 256 + threadIdx.x] = r;
}

template <int OP>
float run(uint32_t* d, int blocks) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
    probe<OP><<<blocks, 256>>>(d, 1);
    (void)hipEventRecord(e0);
    probe<OP><<<blocks, 256>>>(d, 2);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    return ms;
}

int main() {
    int dev = 0; hipDeviceProp_t p; (void)hipGetDeviceProperties(&p, dev);
    const int blocks = p.multiProcessorCount * 8;   // 8 blocks x 4 waves per CU
    uint32_t* d; (void)hipMalloc(&d, (size_t)blocks * 256 * 4);
    const double waves = (double)blocks * 4, ops = (double)N_ITER * 8;
    const double simds = p.multiProcessorCount * 4.0, ghz = p.clockRate * 1e-6;
    const char* names[] = {"v_fma_f32", "v_mul_lo_u32", "v_mad_u32_u24(+add)", "v_rcp_f32", "v_add+v_sqrt_f32", "v_mad_u64_u32(+shift)"};
    float t[6] = {run<0>(d, blocks), run<1>(d, blocks), run<2>(d, blocks), run<3>(d, blocks), run<4>(d, blocks), run<5>(d, blocks)};
    for (int k = 0; k < 6; ++k) {
        // cycles per wave-op on one SIMD = time x clock x SIMDs / (waves x ops)
        double cyc = t[k] * 1e-3 * ghz * 1e9 * simds / (waves * ops);
        printf("{\"op\": \"%s\", \"ms\": %.3f, \"cycles_per_wave_op\": %.2f, \"clock_ghz\": %.2f}\n", names[k], t[k], cyc, ghz);
    }
    (void)hipFree(d);
    return 0;
}
