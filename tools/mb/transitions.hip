// Microbenchmark: cost of VALU->SALU->VALU dependency round trips on gfx950, one game-like
// wave per workgroup; compares a pure-VALU dependent chain, a pure-SALU chain and a chain
// that bounces through v_readfirstlane / v_readlane into scalar code and back.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template <int MODE>
__global__ __launch_bounds__(64) void chain(int iters, unsigned *out, unsigned long long *cyc) {
    unsigned v = threadIdx.x;
    unsigned s = 1;
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
    for (int i = 0; i < iters; ++i) {
        if (MODE == 0) {  // 4 dependent VALU
            v = v * 3u + 1u; v ^= v >> 7; v += 5u; v = v * 7u;
        } else if (MODE == 1) {  // VALU -> readfirstlane -> SALU -> VALU
            v = v * 3u + 1u;
            s = __builtin_amdgcn_readfirstlane(v);
            s = s * 5u + 3u;
            v = v + s;
        } else if (MODE == 2) {  // VALU -> ballot -> SALU ff1 -> readlane(lane=SGPR) -> VALU
            v = v * 3u + 1u;
            unsigned long long b = __ballot(v & 1u);
            int l = __builtin_ctzll(b | (1ull << 63));
            s = __builtin_amdgcn_readlane(v, l);
            v = v + s;
        } else if (MODE == 3) {  // DPP chain
            v = v * 3u + 1u;
            v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xF, 0xF, false);
            v += (unsigned)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xF, 0xF, false);
            v += 5u;
        } else if (MODE == 4) {  // LDS round trip via bpermute
            v = v * 3u + 1u;
            v = (unsigned)__builtin_amdgcn_ds_bpermute((int)(((threadIdx.x + 1) & 63) << 2), (int)v);
            v += 5u;
        }
    }
    const unsigned long long t1 = __builtin_amdgcn_s_memtime();
    out[blockIdx.x * 64 + threadIdx.x] = v + s;
    if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE>
void run(const char *name, int blocks, int iters) {
    unsigned *out; unsigned long long *cyc;
    hipMalloc(&out, blocks * 64 * 4); hipMalloc(&cyc, blocks * 8);
    hipLaunchKernelGGL(chain<MODE>, dim3(blocks), dim3(64), 0, 0, iters, out, cyc);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(blocks);
    hipMemcpy(h.data(), cyc, blocks * 8, hipMemcpyDeviceToHost);
    double avg = 0; for (auto x : h) avg += x; avg /= blocks;
    printf("%-28s blocks %6d  cycles/iter %.1f\n", name, blocks, avg / iters);
    hipFree(out); hipFree(cyc);
}

int main() {
    for (int blocks : {256, 4096, 16384}) {
        run<0>("4 dependent VALU", blocks, 20000);
        run<1>("VALU->rfl->SALU->VALU", blocks, 20000);
        run<2>("VALU->ballot->ff1->readlane", blocks, 20000);
        run<3>("VALU + 2 dependent DPP + VALU", blocks, 20000);
        run<4>("VALU + bpermute + VALU", blocks, 20000);
    }
    return 0;
}
