// What gfx950's f32 -> f16 conversions do with an out-of-range value, with the MODE register's
// FP16_OVFL bit (bit 23) as the kernel starts and cleared (the split planes' range guard).
// Prints MODE and the fp16 bits of f16(1e5), f16(-1e5), f16(65519), f16(65520) through the packed
// (v_cvt_pk_f16_f32) and scalar (v_cvt_f16_f32) conversions.
// Build: hipcc --offload-arch=gfx950 -O3 -o f16_ovfl f16_ovfl.hip
#include <hip/hip_runtime.h>
#include <cstdio>

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

__global__ void k_probe(const float* in, unsigned* out, int clear) {
    if (clear) __builtin_amdgcn_s_setreg(0x5C1, 0);  // hwreg(HW_REG_MODE, 23, 1) <- 0
    const unsigned mode = __builtin_amdgcn_s_getreg(0xF801);  // hwreg(HW_REG_MODE, 0, 32)
    if (threadIdx.x == 0) out[0] = mode;
    for (int i = 0; i < 4; ++i) {
        const float v = in[i];
        unsigned pk;
        asm volatile("v_cvt_pk_f16_f32 %0, %1, %2" : "=v"(pk) : "v"(v), "v"(v));           // packed
        const h2 p = __builtin_bit_cast(h2, pk);
        _Float16 s;
        asm volatile("v_cvt_f16_f32 %0, %1" : "=v"(s) : "v"(v));                            // scalar
        if (threadIdx.x == 0) {
            out[1 + 2 * i] = __builtin_bit_cast(unsigned short, p.x);
            out[2 + 2 * i] = __builtin_bit_cast(unsigned short, s);
        }
    }
}

int main() {
    const float h[4] = {1e5f, -1e5f, 65519.f, 65520.f};
    float* in; unsigned* out;
    (void)hipMalloc(&in, sizeof h);
    (void)hipMalloc(&out, 64);
    (void)hipMemcpy(in, h, sizeof h, hipMemcpyHostToDevice);
    for (int clear = 0; clear < 2; ++clear) {
        hipLaunchKernelGGL(k_probe, dim3(1), dim3(64), 0, 0, in, out, clear);
        unsigned r[9];
        (void)hipMemcpy(r, out, sizeof r, hipMemcpyDeviceToHost);
        printf("FP16_OVFL %s: MODE=0x%08x (bit23=%u)\n", clear ? "cleared" : "as launched", r[0], (r[0] >> 23) & 1);
        for (int i = 0; i < 4; ++i)
            printf("  f16(%g): packed 0x%04x scalar 0x%04x%s\n", h[i], r[1 + 2 * i], r[2 + 2 * i],
                   ((r[1 + 2 * i] & 0x7fff) == 0x7c00 || (r[2 + 2 * i] & 0x7fff) == 0x7c00) ? "  (inf)" : "");
    }
    return 0;
}
