// Does gfx950's L2 keep re-written lines (write-back), or does every store reach the fabric?
// (whether a per-block ring that k_trace rewrites stays in L2.)
// Each block owns a region of R bytes and rewrites it `reps` times with 16-B-per-lane stores
// (optionally reading it back after each pass); WRITE_SIZE / FETCH_SIZE per launch against the
// bytes stored (R * blocks * reps) and the region (R * blocks).
// usage: rocprofv3 --pmc WRITE_SIZE -- ubench_l2wb ; rocprofv3 --pmc FETCH_SIZE -- ubench_l2wb
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_l2wb.hip -o scripts/_build/ubench_l2wb
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void __launch_bounds__(256) k_rewrite(uint4* __restrict__ buf, uint32_t region_vec, int reps, int readback,
                                                 uint32_t* __restrict__ sink)
{
    uint4* r = buf + (size_t)blockIdx.x * region_vec;
    uint32_t acc = 0;
    for (int k = 0; k < reps; ++k) {
        for (uint32_t i = threadIdx.x; i < region_vec; i += blockDim.x) r[i] = make_uint4(i, k, blockIdx.x, 7u);
        if (readback) {
            __builtin_amdgcn_s_waitcnt(0);
            __syncthreads();
            // another lane's store: read back through L2 (L1 bypass)
            for (uint32_t i = threadIdx.x; i < region_vec; i += blockDim.x) {
                typedef uint32_t v4u __attribute__((ext_vector_type(4)));
                v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(r + (region_vec - 1 - i)));
                acc ^= v.x ^ v.y;
            }
            __syncthreads();
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main()
{
    const int blocks = 256;
    uint4* buf;
    uint32_t* sink;
    const size_t max_region = 256 << 10;
    (void)hipMalloc(&buf, max_region * blocks);
    (void)hipMalloc(&sink, 64);
    (void)hipMemset(buf, 0, max_region * blocks);
    (void)hipDeviceSynchronize();
    int launch = 0;
    for (int readback = 0; readback < 2; ++readback)
        for (size_t region : {4096ul, 16384ul, 65536ul, 262144ul}) {
            const int reps = 64;
            hipLaunchKernelGGL(k_rewrite, dim3(blocks), dim3(256), 0, 0, buf, (uint32_t)(region / 16), reps, readback,
                               sink);
            (void)hipDeviceSynchronize();
            printf("launch %2d region %6zu B/block readback %d: stored %.1f MiB, region total %.2f MiB\n", launch++,
                   region, readback, (double)region * blocks * reps / 1048576.0, (double)region * blocks / 1048576.0);
        }
    return 0;
}
