// Microbenchmark: dependent-chain latency per instruction on gfx950 (one wave per CU):
// each iteration issues 8 dependent copies of one instruction (inline asm) + loop control.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

#define R8(x) x x x x x x x x
template <int MODE>
__global__ __launch_bounds__(64) void chain(int iters, unsigned *out, unsigned long long *cyc) {
    unsigned v = threadIdx.x, w = threadIdx.x * 7u + 1u;
    unsigned long long d = threadIdx.x;
    unsigned s = 3;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) asm volatile(R8("v_add_u32 %0, %0, %1\n") : "+v"(v) : "v"(w));
        if (MODE == 1) asm volatile(R8("v_lshrrev_b64 %0, 1, %0\n") : "+v"(d));
        if (MODE == 2) asm volatile(R8("v_mul_u32_u24 %0, %0, %1\n") : "+v"(v) : "v"(w));
        if (MODE == 3) asm volatile(R8("v_mul_lo_u32 %0, %0, %1\n") : "+v"(v) : "v"(w));
        if (MODE == 4) asm volatile(R8("v_bcnt_u32_b32 %0, %0, %1\n") : "+v"(v) : "v"(w));
        if (MODE == 5) asm volatile(R8("v_add_u32_dpp %0, %0, %0 row_shr:1 bound_ctrl:0\n s_nop 1\n") : "+v"(v));
        if (MODE == 6) asm volatile(R8("v_readfirstlane_b32 %1, %0\n v_add_u32 %0, %1, %0\n") : "+v"(v), "+s"(s));
        if (MODE == 7) asm volatile(R8("v_cmp_gt_u32 vcc, %0, %1\n v_cndmask_b32 %0, %0, %1, vcc\n") : "+v"(v) : "v"(w) : "vcc");
        if (MODE == 9) asm volatile(R8("v_add_u32 %0, %0, %1\n s_nop 0\n") : "+v"(v) : "v"(w));
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = v + s + (unsigned)d;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char *name, int blocks, int iters) {
    unsigned *out; unsigned long long *cyc;
    (void)hipMalloc(&out, blocks * 64 * 4); (void)hipMalloc(&cyc, blocks * 8);
    hipLaunchKernelGGL(chain<MODE>, dim3(blocks), dim3(64), 0, 0, iters, out, cyc);
    (void)hipDeviceSynchronize();
    std::vector<unsigned long long> h(blocks);
    (void)hipMemcpy(h.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (auto x : h) avg += x; avg /= blocks;
    printf("%-34s blocks %6d  cycles per dependent instruction %.2f\n", name, blocks, avg / iters / 8);
    (void)hipFree(out); (void)hipFree(cyc);
}

int main() {
    for (int blocks : {256, 1024, 4096}) {
        run<0>("v_add_u32", blocks, 20000);
        run<1>("v_lshrrev_b64", blocks, 20000);
        run<2>("v_mul_u32_u24", blocks, 20000);
        run<3>("v_mul_lo_u32", blocks, 20000);
        run<4>("v_bcnt_u32_b32", blocks, 20000);
        run<5>("v_add_u32_dpp row_shr + s_nop 1", blocks, 20000);
        run<6>("v_readfirstlane + v_add (pair)", blocks, 20000);
        run<7>("v_cmp -> vcc + v_cndmask (pair)", blocks, 20000);
        run<9>("v_add_u32 + s_nop 0 (pair)", blocks, 20000);
    }
    return 0;
}
