#include <hip/hip_runtime.h>
template <int J> __device__ __forceinline__ unsigned shx(unsigned v) {
    const unsigned lane = threadIdx.x & 63;
    if constexpr (J == 1) return __builtin_amdgcn_mov_dpp(v, 0xB1, 0xF, 0xF, false);
    else if constexpr (J == 2) return __builtin_amdgcn_mov_dpp(v, 0x4E, 0xF, 0xF, false);
    else if constexpr (J == 4) return __builtin_amdgcn_mov_dpp(__builtin_amdgcn_mov_dpp(v, 0x141, 0xF, 0xF, false), 0x1B, 0xF, 0xF, false);
    else if constexpr (J == 8) return __builtin_amdgcn_mov_dpp(v, 0x128, 0xF, 0xF, false);
    else if constexpr (J == 16) { auto p = __builtin_amdgcn_permlane16_swap(v, v, false, false); return (lane & 16) ? p[0] : p[1]; }
    else { auto p = __builtin_amdgcn_permlane32_swap(v, v, false, false); return (lane & 32) ? p[0] : p[1]; }
}
__global__ void k(unsigned* out) {
    const unsigned v = threadIdx.x;
    out[threadIdx.x * 6 + 0] = shx<1>(v); out[threadIdx.x * 6 + 1] = shx<2>(v); out[threadIdx.x * 6 + 2] = shx<4>(v);
    out[threadIdx.x * 6 + 3] = shx<8>(v); out[threadIdx.x * 6 + 4] = shx<16>(v); out[threadIdx.x * 6 + 5] = shx<32>(v);
}
int main() {
    unsigned* d; hipMalloc(&d, 64 * 6 * 4); hipLaunchKernelGGL(k, 1, 64, 0, 0, d);
    unsigned h[64 * 6]; hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int bad = 0; const int J[6] = {1, 2, 4, 8, 16, 32};
    for (int l = 0; l < 64; l++) for (int k = 0; k < 6; k++) if (h[l * 6 + k] != (unsigned)(l ^ J[k])) { if (bad < 10) printf("lane %d xor %d got %u\n", l, J[k], h[l*6+k]); bad++; }
    printf("shx check: %d bad\n", bad); return bad != 0;
}
