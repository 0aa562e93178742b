// Does a device-scope global atomic on gfx950 stay in the XCD's L2, or does each one reach HBM?
// (the AO-count atomics of C5 cost ~74 MiB of WRITE_SIZE per 4K frame.)
// Launches, each 256 blocks x 256 threads, every thread `reps` operations:
//   0: atomicAdd (no return) on its block's 4 KiB region (the words stay hot in L2)
//   1: atomicAdd (no return) on a random word of a 32 MiB array (the AO-count pattern)
//   2: plain 4-B stores to the same random words
//   3: atomicAdd with return on random words
// WRITE_SIZE / FETCH_SIZE per launch against the operation count x 4 B.
// usage: rocprofv3 --pmc WRITE_SIZE -- ubench_atomic ; rocprofv3 --pmc FETCH_SIZE -- ubench_atomic
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_atomic.hip -o scripts/_build/ubench_atomic
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__global__ void __launch_bounds__(256) k_op(uint32_t* __restrict__ buf, uint32_t words, int mode, int reps,
                                            uint32_t* __restrict__ sink)
{
    uint32_t x = blockIdx.x * 256u + threadIdx.x + 1u, acc = 0;
    for (int k = 0; k < reps; ++k) {
        x ^= x << 13;
        x ^= x >> 17;
        x ^= x << 5;
        if (mode == 0) {
            atomicAdd(buf + (size_t)blockIdx.x * 1024u + (x & 1023u), 1u);
        } else {
            uint32_t* p = buf + (x % words);
            if (mode == 1) atomicAdd(p, 1u);
            else if (mode == 2) *p = x;
            else acc += atomicAdd(p, 1u);
        }
    }
    if (acc == 0x12345678u) sink[0] = acc;
}

int main()
{
    const int blocks = 256, reps = 64;
    const uint32_t words = 8u << 20; // 32 MiB
    uint32_t *buf, *sink;
    (void)hipMalloc(&buf, (size_t)words * 4);
    (void)hipMalloc(&sink, 64);
    (void)hipMemset(buf, 0, (size_t)words * 4);
    (void)hipDeviceSynchronize();
    const char* names[] = {"atomicAdd, 4 KiB per block", "atomicAdd, random in 32 MiB", "store, random in 32 MiB",
                           "atomicAdd with return, random in 32 MiB"};
    for (int mode = 0; mode < 4; ++mode) {
        hipLaunchKernelGGL(k_op, dim3(blocks), dim3(256), 0, 0, buf, words, mode, reps, sink);
        (void)hipDeviceSynchronize();
        printf("launch %d %-40s: %d ops = %.2f MiB of 4-B operands\n", mode, names[mode], blocks * 256 * reps,
               (double)blocks * 256 * reps * 4 / 1048576.0);
    }
    return 0;
}
