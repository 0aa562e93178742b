// VGPR bank conflicts on gfx950: issue cost of v_fma_f32 / v_pk_fma_f32 / v_add_f32 streams whose
// source operands sit in distinct or equal register banks (bank = VGPR index mod 4), 8 independent
// chains per lane, 4 waves per SIMD.  Registers are pinned by explicit asm operands.
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_bank.hip -o scripts/_build/ubench_bank
#include <hip/hip_runtime.h>

#include <cstdio>

constexpr int kIters = 2048;

// 8 chains: destination/accumulator in v[40 + 4i .. ] so the operand banks are chosen by the
// instruction text.  Chain i accumulates in VGPR (40 + 4*i) (bank 0); sources in v32..v39.
#define R8(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7)

template <int K>
__global__ void __launch_bounds__(1024) k_bank(float* out, unsigned long long* clk)
{
    __shared__ float lds_pad[4096 + 64 * 4];
    if (threadIdx.x < 64) lds_pad[threadIdx.x] = 0.0f;
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    const float x = (float)threadIdx.x * 1e-9f;
    asm volatile(
        "v_mov_b32 v32, %0\n v_mov_b32 v33, %0\n v_mov_b32 v34, %0\n v_mov_b32 v35, %0\n"
        "v_mov_b32 v36, %0\n v_mov_b32 v37, %0\n v_mov_b32 v38, %0\n v_mov_b32 v39, %0\n"
        "v_mov_b32 v40, %0\n v_mov_b32 v44, %0\n v_mov_b32 v48, %0\n v_mov_b32 v52, %0\n"
        "v_mov_b32 v56, %0\n v_mov_b32 v60, %0\n v_mov_b32 v64, %0\n v_mov_b32 v68, %0\n"
        "v_mov_b32 v41, %0\n v_mov_b32 v45, %0\n v_mov_b32 v49, %0\n v_mov_b32 v53, %0\n"
        "v_mov_b32 v57, %0\n v_mov_b32 v61, %0\n v_mov_b32 v65, %0\n v_mov_b32 v69, %0\n"
        :: "v"(x) : "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v44", "v45", "v48",
        "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
    const unsigned int laddr = (threadIdx.x & 63u) * 16u;
    for (int it = 0; it < kIters; ++it) {
        if constexpr (K == 0) // acc bank 0, sources banks 1 and 2: no conflict
            asm volatile("v_fma_f32 v40, v40, v33, v34\n v_fma_f32 v44, v44, v33, v34\n v_fma_f32 v48, v48, v33, v34\n v_fma_f32 v52, v52, v33, v34\n"
                         "v_fma_f32 v56, v56, v33, v34\n v_fma_f32 v60, v60, v33, v34\n v_fma_f32 v64, v64, v33, v34\n v_fma_f32 v68, v68, v33, v34\n"
                         ::: "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68");
        if constexpr (K == 1) // acc bank 0, one source bank 0
            asm volatile("v_fma_f32 v40, v40, v32, v34\n v_fma_f32 v44, v44, v32, v34\n v_fma_f32 v48, v48, v32, v34\n v_fma_f32 v52, v52, v32, v34\n"
                         "v_fma_f32 v56, v56, v32, v34\n v_fma_f32 v60, v60, v32, v34\n v_fma_f32 v64, v64, v32, v34\n v_fma_f32 v68, v68, v32, v34\n"
                         ::: "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68");
        if constexpr (K == 2) // all three operands bank 0
            asm volatile("v_fma_f32 v40, v40, v32, v36\n v_fma_f32 v44, v44, v32, v36\n v_fma_f32 v48, v48, v32, v36\n v_fma_f32 v52, v52, v32, v36\n"
                         "v_fma_f32 v56, v56, v32, v36\n v_fma_f32 v60, v60, v32, v36\n v_fma_f32 v64, v64, v32, v36\n v_fma_f32 v68, v68, v32, v36\n"
                         ::: "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68");
        if constexpr (K == 3) // two sources, distinct banks (v_add)
            asm volatile("v_add_f32 v40, v40, v33\n v_add_f32 v44, v44, v33\n v_add_f32 v48, v48, v33\n v_add_f32 v52, v52, v33\n"
                         "v_add_f32 v56, v56, v33\n v_add_f32 v60, v60, v33\n v_add_f32 v64, v64, v33\n v_add_f32 v68, v68, v33\n"
                         ::: "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68");
        if constexpr (K == 4) // two sources, same bank (v_add)
            asm volatile("v_add_f32 v40, v40, v32\n v_add_f32 v44, v44, v32\n v_add_f32 v48, v48, v32\n v_add_f32 v52, v52, v32\n"
                         "v_add_f32 v56, v56, v32\n v_add_f32 v60, v60, v32\n v_add_f32 v64, v64, v32\n v_add_f32 v68, v68, v32\n"
                         ::: "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68");
        if constexpr (K == 5) // pk_fma: acc v[40:41] banks 0,1; sources v[34:35] banks 2,3 and v[38:39] banks 2,3
            asm volatile("v_pk_fma_f32 v[40:41], v[40:41], v[34:35], v[38:39]\n v_pk_fma_f32 v[44:45], v[44:45], v[34:35], v[38:39]\n"
                         "v_pk_fma_f32 v[48:49], v[48:49], v[34:35], v[38:39]\n v_pk_fma_f32 v[52:53], v[52:53], v[34:35], v[38:39]\n"
                         "v_pk_fma_f32 v[56:57], v[56:57], v[34:35], v[38:39]\n v_pk_fma_f32 v[60:61], v[60:61], v[34:35], v[38:39]\n"
                         "v_pk_fma_f32 v[64:65], v[64:65], v[34:35], v[38:39]\n v_pk_fma_f32 v[68:69], v[68:69], v[34:35], v[38:39]\n"
                         ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 6) // pk_fma, all sources banks 0,1
            asm volatile("v_pk_fma_f32 v[40:41], v[40:41], v[32:33], v[36:37]\n v_pk_fma_f32 v[44:45], v[44:45], v[32:33], v[36:37]\n"
                         "v_pk_fma_f32 v[48:49], v[48:49], v[32:33], v[36:37]\n v_pk_fma_f32 v[52:53], v[52:53], v[32:33], v[36:37]\n"
                         "v_pk_fma_f32 v[56:57], v[56:57], v[32:33], v[36:37]\n v_pk_fma_f32 v[60:61], v[60:61], v[32:33], v[36:37]\n"
                         "v_pk_fma_f32 v[64:65], v[64:65], v[32:33], v[36:37]\n v_pk_fma_f32 v[68:69], v[68:69], v[32:33], v[36:37]\n"
                         ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 7) // pk_mul with op_sel_hi broadcast of a scalar lane (as the noise body): acc x bank-2 pair
            asm volatile("v_pk_mul_f32 v[40:41], v[40:41], v[34:35] op_sel_hi:[1,0]\n v_pk_mul_f32 v[44:45], v[44:45], v[34:35] op_sel_hi:[1,0]\n"
                         "v_pk_mul_f32 v[48:49], v[48:49], v[34:35] op_sel_hi:[1,0]\n v_pk_mul_f32 v[52:53], v[52:53], v[34:35] op_sel_hi:[1,0]\n"
                         "v_pk_mul_f32 v[56:57], v[56:57], v[34:35] op_sel_hi:[1,0]\n v_pk_mul_f32 v[60:61], v[60:61], v[34:35] op_sel_hi:[1,0]\n"
                         "v_pk_mul_f32 v[64:65], v[64:65], v[34:35] op_sel_hi:[1,0]\n v_pk_mul_f32 v[68:69], v[68:69], v[34:35] op_sel_hi:[1,0]\n"
                         ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 8) // fma with an SGPR source and a literal-free VGPR (1 VGPR read besides acc)
            asm volatile("v_fma_f32 v40, v40, s0, v33\n v_fma_f32 v44, v44, s0, v33\n v_fma_f32 v48, v48, s0, v33\n v_fma_f32 v52, v52, s0, v33\n"
                         "v_fma_f32 v56, v56, s0, v33\n v_fma_f32 v60, v60, s0, v33\n v_fma_f32 v64, v64, s0, v33\n v_fma_f32 v68, v68, s0, v33\n"
                         ::: "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68");
        if constexpr (K == 9) // v_fma acc b0, v33, v33 (same reg twice)
            asm volatile("v_fma_f32 v40, v40, v33, v33\n v_fma_f32 v44, v44, v33, v33\n v_fma_f32 v48, v48, v33, v33\n v_fma_f32 v52, v52, v33, v33\n v_fma_f32 v56, v56, v33, v33\n v_fma_f32 v60, v60, v33, v33\n v_fma_f32 v64, v64, v33, v33\n v_fma_f32 v68, v68, v33, v33\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 10) // v_fma acc b0, v33, 2.0 (inline const)
            asm volatile("v_fma_f32 v40, v40, v33, 2.0\n v_fma_f32 v44, v44, v33, 2.0\n v_fma_f32 v48, v48, v33, 2.0\n v_fma_f32 v52, v52, v33, 2.0\n v_fma_f32 v56, v56, v33, 2.0\n v_fma_f32 v60, v60, v33, 2.0\n v_fma_f32 v64, v64, v33, 2.0\n v_fma_f32 v68, v68, v33, 2.0\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 11) // v_fmac acc b0 += v33*v34
            asm volatile("v_fmac_f32 v40, v33, v34\n v_fmac_f32 v44, v33, v34\n v_fmac_f32 v48, v33, v34\n v_fmac_f32 v52, v33, v34\n v_fmac_f32 v56, v33, v34\n v_fmac_f32 v60, v33, v34\n v_fmac_f32 v64, v33, v34\n v_fmac_f32 v68, v33, v34\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 12) // v_fmac acc b0 += v32*v34 (src b0)
            asm volatile("v_fmac_f32 v40, v32, v34\n v_fmac_f32 v44, v32, v34\n v_fmac_f32 v48, v32, v34\n v_fmac_f32 v52, v32, v34\n v_fmac_f32 v56, v32, v34\n v_fmac_f32 v60, v32, v34\n v_fmac_f32 v64, v32, v34\n v_fmac_f32 v68, v32, v34\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 13) // v_fmamk acc b0 = acc*K + v33
            asm volatile("v_fmamk_f32 v40, v40, 0x3f800001, v33\n v_fmamk_f32 v44, v44, 0x3f800001, v33\n v_fmamk_f32 v48, v48, 0x3f800001, v33\n v_fmamk_f32 v52, v52, 0x3f800001, v33\n v_fmamk_f32 v56, v56, 0x3f800001, v33\n v_fmamk_f32 v60, v60, 0x3f800001, v33\n v_fmamk_f32 v64, v64, 0x3f800001, v33\n v_fmamk_f32 v68, v68, 0x3f800001, v33\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 14) // v_fma acc b0, v33, s0 (sgpr src2)
            asm volatile("v_fma_f32 v40, v40, v33, s0\n v_fma_f32 v44, v44, v33, s0\n v_fma_f32 v48, v48, v33, s0\n v_fma_f32 v52, v52, v33, s0\n v_fma_f32 v56, v56, v33, s0\n v_fma_f32 v60, v60, v33, s0\n v_fma_f32 v64, v64, v33, s0\n v_fma_f32 v68, v68, v33, s0\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 15) // v_fma acc b0, v33, v37 (2 srcs in b1)
            asm volatile("v_fma_f32 v40, v40, v33, v37\n v_fma_f32 v44, v44, v33, v37\n v_fma_f32 v48, v48, v33, v37\n v_fma_f32 v52, v52, v33, v37\n v_fma_f32 v56, v56, v33, v37\n v_fma_f32 v60, v60, v33, v37\n v_fma_f32 v64, v64, v33, v37\n v_fma_f32 v68, v68, v33, v37\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 16) // v_perm acc b0, v33, v34 (3 vgpr banks)
            asm volatile("v_perm_b32 v40, v40, v33, v34\n v_perm_b32 v44, v44, v33, v34\n v_perm_b32 v48, v48, v33, v34\n v_perm_b32 v52, v52, v33, v34\n v_perm_b32 v56, v56, v33, v34\n v_perm_b32 v60, v60, v33, v34\n v_perm_b32 v64, v64, v33, v34\n v_perm_b32 v68, v68, v33, v34\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 17) // v_perm acc b0, v33, s0
            asm volatile("v_perm_b32 v40, v40, v33, s0\n v_perm_b32 v44, v44, v33, s0\n v_perm_b32 v48, v48, v33, s0\n v_perm_b32 v52, v52, v33, s0\n v_perm_b32 v56, v56, v33, s0\n v_perm_b32 v60, v60, v33, s0\n v_perm_b32 v64, v64, v33, s0\n v_perm_b32 v68, v68, v33, s0\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 18) // v_floor acc
            asm volatile("v_floor_f32 v40, v40\n v_floor_f32 v44, v44\n v_floor_f32 v48, v48\n v_floor_f32 v52, v52\n v_floor_f32 v56, v56\n v_floor_f32 v60, v60\n v_floor_f32 v64, v64\n v_floor_f32 v68, v68\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 19) // v_lshl_or acc b0, 9, v33
            asm volatile("v_lshl_or_b32 v40, v40, 9, v33\n v_lshl_or_b32 v44, v44, 9, v33\n v_lshl_or_b32 v48, v48, 9, v33\n v_lshl_or_b32 v52, v52, 9, v33\n v_lshl_or_b32 v56, v56, 9, v33\n v_lshl_or_b32 v60, v60, 9, v33\n v_lshl_or_b32 v64, v64, 9, v33\n v_lshl_or_b32 v68, v68, 9, v33\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 20) // v_lshl_or acc b0, v34, v33
            asm volatile("v_lshl_or_b32 v40, v40, v34, v33\n v_lshl_or_b32 v44, v44, v34, v33\n v_lshl_or_b32 v48, v48, v34, v33\n v_lshl_or_b32 v52, v52, v34, v33\n v_lshl_or_b32 v56, v56, v34, v33\n v_lshl_or_b32 v60, v60, v34, v33\n v_lshl_or_b32 v64, v64, v34, v33\n v_lshl_or_b32 v68, v68, v34, v33\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 21) // v_and_or acc b0, v33, v34
            asm volatile("v_and_or_b32 v40, v40, v33, v34\n v_and_or_b32 v44, v44, v33, v34\n v_and_or_b32 v48, v48, v33, v34\n v_and_or_b32 v52, v52, v33, v34\n v_and_or_b32 v56, v56, v33, v34\n v_and_or_b32 v60, v60, v33, v34\n v_and_or_b32 v64, v64, v33, v34\n v_and_or_b32 v68, v68, v33, v34\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 22) // v_pk_add acc b01, v[34:35]
            asm volatile("v_pk_add_f32 v[40:41], v[40:41], v[34:35]\n v_pk_add_f32 v[44:45], v[44:45], v[34:35]\n v_pk_add_f32 v[48:49], v[48:49], v[34:35]\n v_pk_add_f32 v[52:53], v[52:53], v[34:35]\n v_pk_add_f32 v[56:57], v[56:57], v[34:35]\n v_pk_add_f32 v[60:61], v[60:61], v[34:35]\n v_pk_add_f32 v[64:65], v[64:65], v[34:35]\n v_pk_add_f32 v[68:69], v[68:69], v[34:35]\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 23) // v_pk_fma acc, v[34:35], s[0:1]
            asm volatile("v_pk_fma_f32 v[40:41], v[40:41], v[34:35], s[0:1] op_sel_hi:[1,1,0]\n v_pk_fma_f32 v[44:45], v[44:45], v[34:35], s[0:1] op_sel_hi:[1,1,0]\n v_pk_fma_f32 v[48:49], v[48:49], v[34:35], s[0:1] op_sel_hi:[1,1,0]\n v_pk_fma_f32 v[52:53], v[52:53], v[34:35], s[0:1] op_sel_hi:[1,1,0]\n v_pk_fma_f32 v[56:57], v[56:57], v[34:35], s[0:1] op_sel_hi:[1,1,0]\n v_pk_fma_f32 v[60:61], v[60:61], v[34:35], s[0:1] op_sel_hi:[1,1,0]\n v_pk_fma_f32 v[64:65], v[64:65], v[34:35], s[0:1] op_sel_hi:[1,1,0]\n v_pk_fma_f32 v[68:69], v[68:69], v[34:35], s[0:1] op_sel_hi:[1,1,0]\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 24) // v_mul acc b0, v33
            asm volatile("v_mul_f32 v40, v40, v33\n v_mul_f32 v44, v44, v33\n v_mul_f32 v48, v48, v33\n v_mul_f32 v52, v52, v33\n v_mul_f32 v56, v56, v33\n v_mul_f32 v60, v60, v33\n v_mul_f32 v64, v64, v33\n v_mul_f32 v68, v68, v33\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 25) // v_sub acc b0, v33, acc (VOP2 rev)
            asm volatile("v_sub_f32 v40, v33, v40\n v_sub_f32 v44, v33, v44\n v_sub_f32 v48, v33, v48\n v_sub_f32 v52, v33, v52\n v_sub_f32 v56, v33, v56\n v_sub_f32 v60, v33, v60\n v_sub_f32 v64, v33, v64\n v_sub_f32 v68, v33, v68\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 26) // v_mad_u32_u24 acc, v33, v34
            asm volatile("v_mad_u32_u24 v40, v40, v33, v34\n v_mad_u32_u24 v44, v44, v33, v34\n v_mad_u32_u24 v48, v48, v33, v34\n v_mad_u32_u24 v52, v52, v33, v34\n v_mad_u32_u24 v56, v56, v33, v34\n v_mad_u32_u24 v60, v60, v33, v34\n v_mad_u32_u24 v64, v64, v33, v34\n v_mad_u32_u24 v68, v68, v33, v34\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 27) // v_fma acc b0, v33, v38 (b1,b2)
            asm volatile("v_fma_f32 v40, v40, v33, v38\n v_fma_f32 v44, v44, v33, v38\n v_fma_f32 v48, v48, v33, v38\n v_fma_f32 v52, v52, v33, v38\n v_fma_f32 v56, v56, v33, v38\n v_fma_f32 v60, v60, v33, v38\n v_fma_f32 v64, v64, v33, v38\n v_fma_f32 v68, v68, v33, v38\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 28) // v_fma acc b0, v35, v34 (b3,b2)
            asm volatile("v_fma_f32 v40, v40, v35, v34\n v_fma_f32 v44, v44, v35, v34\n v_fma_f32 v48, v48, v35, v34\n v_fma_f32 v52, v52, v35, v34\n v_fma_f32 v56, v56, v35, v34\n v_fma_f32 v60, v60, v35, v34\n v_fma_f32 v64, v64, v35, v34\n v_fma_f32 v68, v68, v35, v34\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 29) // v_cvt_i32_f32 acc
            asm volatile("v_cvt_i32_f32 v40, v40\n v_cvt_i32_f32 v44, v44\n v_cvt_i32_f32 v48, v48\n v_cvt_i32_f32 v52, v52\n v_cvt_i32_f32 v56, v56\n v_cvt_i32_f32 v60, v60\n v_cvt_i32_f32 v64, v64\n v_cvt_i32_f32 v68, v68\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 30) // v_and_b32 acc, 0x7f7f (literal)
            asm volatile("v_and_b32 v40, 0x7f7f7f7f, v40\n v_and_b32 v44, 0x7f7f7f7f, v44\n v_and_b32 v48, 0x7f7f7f7f, v48\n v_and_b32 v52, 0x7f7f7f7f, v52\n v_and_b32 v56, 0x7f7f7f7f, v56\n v_and_b32 v60, 0x7f7f7f7f, v60\n v_and_b32 v64, 0x7f7f7f7f, v64\n v_and_b32 v68, 0x7f7f7f7f, v68\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 31) // v_add acc, literal
            asm volatile("v_add_f32 v40, 0x4b400000, v40\n v_add_f32 v44, 0x4b400000, v44\n v_add_f32 v48, 0x4b400000, v48\n v_add_f32 v52, 0x4b400000, v52\n v_add_f32 v56, 0x4b400000, v56\n v_add_f32 v60, 0x4b400000, v60\n v_add_f32 v64, 0x4b400000, v64\n v_add_f32 v68, 0x4b400000, v68\n " ::: "v40", "v41", "v44", "v45", "v48", "v49", "v52", "v53", "v56", "v57", "v60", "v61", "v64", "v65", "v68", "v69");
        if constexpr (K == 40) // 8 fma (no conflict) + 0 LDS
            asm volatile("v_fma_f32 v40, v40, v33, v34\n v_fma_f32 v44, v44, v33, v34\n v_fma_f32 v48, v48, v33, v34\n v_fma_f32 v52, v52, v33, v34\n v_fma_f32 v56, v56, v33, v34\n v_fma_f32 v60, v60, v33, v34\n v_fma_f32 v64, v64, v33, v34\n v_fma_f32 v68, v68, v33, v34\n s_waitcnt lgkmcnt(0)\n " :: "v"(laddr) : "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107");
        if constexpr (K == 41) // 8 fma + 1 ds_read_b128
            asm volatile("ds_read_b128 v[92:95], v90\n v_fma_f32 v40, v40, v33, v34\n v_fma_f32 v44, v44, v33, v34\n v_fma_f32 v48, v48, v33, v34\n v_fma_f32 v52, v52, v33, v34\n v_fma_f32 v56, v56, v33, v34\n v_fma_f32 v60, v60, v33, v34\n v_fma_f32 v64, v64, v33, v34\n v_fma_f32 v68, v68, v33, v34\n s_waitcnt lgkmcnt(0)\n " :: "v"(laddr) : "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107");
        if constexpr (K == 42) // 8 fma + 2 ds_read_b128
            asm volatile("ds_read_b128 v[92:95], v90\n ds_read_b128 v[96:99], v90 offset:1024\n v_fma_f32 v40, v40, v33, v34\n v_fma_f32 v44, v44, v33, v34\n v_fma_f32 v48, v48, v33, v34\n v_fma_f32 v52, v52, v33, v34\n v_fma_f32 v56, v56, v33, v34\n v_fma_f32 v60, v60, v33, v34\n v_fma_f32 v64, v64, v33, v34\n v_fma_f32 v68, v68, v33, v34\n s_waitcnt lgkmcnt(0)\n " :: "v"(laddr) : "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107");
        if constexpr (K == 43) // 8 fma + 4 ds_read_b128
            asm volatile("ds_read_b128 v[92:95], v90\n ds_read_b128 v[96:99], v90 offset:1024\n ds_read_b128 v[100:103], v90 offset:2048\n ds_read_b128 v[104:107], v90 offset:3072\n v_fma_f32 v40, v40, v33, v34\n v_fma_f32 v44, v44, v33, v34\n v_fma_f32 v48, v48, v33, v34\n v_fma_f32 v52, v52, v33, v34\n v_fma_f32 v56, v56, v33, v34\n v_fma_f32 v60, v60, v33, v34\n v_fma_f32 v64, v64, v33, v34\n v_fma_f32 v68, v68, v33, v34\n s_waitcnt lgkmcnt(0)\n " :: "v"(laddr) : "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107");
        if constexpr (K == 44) // 8 fma + 4 ds_read_b64
            asm volatile("ds_read_b64 v[92:93], v90\n ds_read_b64 v[96:97], v90 offset:1024\n ds_read_b64 v[100:101], v90 offset:2048\n ds_read_b64 v[104:105], v90 offset:3072\n v_fma_f32 v40, v40, v33, v34\n v_fma_f32 v44, v44, v33, v34\n v_fma_f32 v48, v48, v33, v34\n v_fma_f32 v52, v52, v33, v34\n v_fma_f32 v56, v56, v33, v34\n v_fma_f32 v60, v60, v33, v34\n v_fma_f32 v64, v64, v33, v34\n v_fma_f32 v68, v68, v33, v34\n s_waitcnt lgkmcnt(0)\n " :: "v"(laddr) : "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107");
        if constexpr (K == 45) // 8 fma + 4 ds_read_b32
            asm volatile("ds_read_b32 v92, v90\n ds_read_b32 v96, v90 offset:1024\n ds_read_b32 v100, v90 offset:2048\n ds_read_b32 v104, v90 offset:3072\n v_fma_f32 v40, v40, v33, v34\n v_fma_f32 v44, v44, v33, v34\n v_fma_f32 v48, v48, v33, v34\n v_fma_f32 v52, v52, v33, v34\n v_fma_f32 v56, v56, v33, v34\n v_fma_f32 v60, v60, v33, v34\n v_fma_f32 v64, v64, v33, v34\n v_fma_f32 v68, v68, v33, v34\n s_waitcnt lgkmcnt(0)\n " :: "v"(laddr) : "v40", "v44", "v48", "v52", "v56", "v60", "v64", "v68", "v92", "v93", "v94", "v95", "v96", "v97", "v98", "v99", "v100", "v101", "v102", "v103", "v104", "v105", "v106", "v107");
    }
    float r;
    asm volatile("v_add_f32 %0, v40, v44\n v_add_f32 %0, %0, v48\n v_add_f32 %0, %0, v68" : "=v"(r));
    out[blockIdx.x * blockDim.x + threadIdx.x] = r;
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        clk[0] = __builtin_amdgcn_s_memtime() - t0;
        clk[1] = __builtin_amdgcn_s_memrealtime() - r0;
    }
}

template <int K>
void run(const char* name, float* out, unsigned long long* clk)
{
    hipLaunchKernelGGL(k_bank<K>, dim3(256), dim3(1024), 0, 0, out, clk);
    (void)hipDeviceSynchronize();
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(k_bank<K>, dim3(256), dim3(1024), 0, 0, out, clk);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, e0, e1);
    unsigned long long c[2];
    (void)hipMemcpy(c, clk, sizeof(c), hipMemcpyDeviceToHost);
    const double ghz = (double)c[0] / ((double)c[1] / 100e6) / 1e9;
    const double per = ms / 5 * 1e-3 / ((double)kIters * 8 * 4);
    printf("%-52s %.2f cycles per wave-instruction per SIMD (clock %.2f GHz)\n", name, per * ghz * 1e9, ghz);
}

int main()
{
    float* out;
    unsigned long long* clk;
    (void)hipMalloc(&out, 256 * 1024 * sizeof(float));
    (void)hipMalloc(&clk, 16);
    run<40>("8 fma (no conflict) + 0 LDS", out, clk);
    run<41>("8 fma + 1 ds_read_b128", out, clk);
    run<42>("8 fma + 2 ds_read_b128", out, clk);
    run<43>("8 fma + 4 ds_read_b128", out, clk);
    run<44>("8 fma + 4 ds_read_b64", out, clk);
    run<45>("8 fma + 4 ds_read_b32", out, clk);
    run<0>("v_fma acc b0, src b1, b2 (distinct banks)", out, clk);
    run<1>("v_fma acc b0, src b0, b2 (2 in bank 0)", out, clk);
    run<2>("v_fma acc b0, src b0, b0 (3 in bank 0)", out, clk);
    run<3>("v_add acc b0, src b1", out, clk);
    run<4>("v_add acc b0, src b0", out, clk);
    run<5>("v_pk_fma acc b01, src b23, b23", out, clk);
    run<6>("v_pk_fma acc b01, src b01, b01", out, clk);
    run<7>("v_pk_mul acc b01, src b23 op_sel_hi broadcast", out, clk);
    run<8>("v_fma acc b0, s0, src b1", out, clk);
    run<9>("v_fma acc b0, v33, v33 (same reg twice)", out, clk);
    run<10>("v_fma acc b0, v33, 2.0 (inline const)", out, clk);
    run<11>("v_fmac acc b0 += v33*v34", out, clk);
    run<12>("v_fmac acc b0 += v32*v34 (src b0)", out, clk);
    run<13>("v_fmamk acc b0 = acc*K + v33", out, clk);
    run<14>("v_fma acc b0, v33, s0 (sgpr src2)", out, clk);
    run<15>("v_fma acc b0, v33, v37 (2 srcs in b1)", out, clk);
    run<16>("v_perm acc b0, v33, v34 (3 vgpr banks)", out, clk);
    run<17>("v_perm acc b0, v33, s0", out, clk);
    run<18>("v_floor acc", out, clk);
    run<19>("v_lshl_or acc b0, 9, v33", out, clk);
    run<20>("v_lshl_or acc b0, v34, v33", out, clk);
    run<21>("v_and_or acc b0, v33, v34", out, clk);
    run<22>("v_pk_add acc b01, v[34:35]", out, clk);
    run<23>("v_pk_fma acc, v[34:35], s[0:1]", out, clk);
    run<24>("v_mul acc b0, v33", out, clk);
    run<25>("v_sub acc b0, v33, acc (VOP2 rev)", out, clk);
    run<26>("v_mad_u32_u24 acc, v33, v34", out, clk);
    run<27>("v_fma acc b0, v33, v38 (b1,b2)", out, clk);
    run<28>("v_fma acc b0, v35, v34 (b3,b2)", out, clk);
    run<29>("v_cvt_i32_f32 acc", out, clk);
    run<30>("v_and_b32 acc, 0x7f7f (literal)", out, clk);
    run<31>("v_add acc, literal", out, clk);
    return 0;
}
