// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths k_trace and
// k_finish use (MI355X_MICROARCH.md: FETCH_SIZE reports half the bytes of a 16-B-per-lane streaming
// read; other widths are uncalibrated).  Each kernel touches a known byte count of a 1 GiB buffer
// (beyond the 256 MiB Infinity Cache, untouched by the kernel before it):
//   read_w{4,8,16}      every lane, contiguous, w bytes per lane
//   read_w{4,8,16}_44   the lanes of 44% of the 64-lane groups (the hit units of C3), contiguous
//   write_w{4,8,16}     every lane, contiguous
//   write_w{4,8,16}_44  44% of the 64-lane groups
// usage: ubench_hbm            -> prints the expected bytes of each launch (in launch order)
//        rocprofv3 --pmc FETCH_SIZE -- ubench_hbm ; rocprofv3 --pmc WRITE_SIZE -- ubench_hbm
// build: hipcc --offload-arch=gfx950 -O3 scripts/ubench_hbm.hip -o scripts/_build/ubench_hbm
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr size_t kBytes = 1ull << 30;

__device__ __forceinline__ bool group_active(size_t i, int sparse)
{
    if (!sparse) return true;
    const uint32_t g = (uint32_t)(i >> 6);
    return (g * 2654435761u >> 24) % 100u < 44u; // 44 of 100 groups, scattered
}

template <int W>
struct Vec;
template <>
struct Vec<4> {
    typedef uint32_t T;
};
template <>
struct Vec<8> {
    typedef uint2 T;
};
template <>
struct Vec<16> {
    typedef uint4 T;
};

__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

template <int W>
__global__ void __launch_bounds__(256) k_read(const typename Vec<W>::T* __restrict__ src, size_t n, int sparse,
                                              uint32_t* __restrict__ sink)
{
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        if (group_active(i, sparse)) acc ^= fold(src[i]);
    if (acc == 0x12345678u) sink[0] = acc; // keeps the loads
}

template <int W>
__global__ void __launch_bounds__(256) k_write(typename Vec<W>::T* __restrict__ dst, size_t n, int sparse)
{
    typename Vec<W>::T v;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        if (!group_active(i, sparse)) continue;
        if constexpr (W == 4) v = (uint32_t)i;
        else if constexpr (W == 8) v = make_uint2((uint32_t)i, 1u);
        else v = make_uint4((uint32_t)i, 1u, 2u, 3u);
        dst[i] = v;
    }
}

static size_t active_elems(size_t n, int sparse)
{
    if (!sparse) return n;
    size_t c = 0;
    for (size_t g = 0; g < n / 64; ++g)
        if (((uint32_t)g * 2654435761u >> 24) % 100u < 44u) c += 64;
    return c;
}

int main()
{
    char* buf[2];
    uint32_t* sink;
    (void)hipMalloc(&buf[0], kBytes);
    (void)hipMalloc(&buf[1], kBytes);
    (void)hipMalloc(&sink, 64);
    // the read buffer holds data written long before (and evicted by the second buffer's fill)
    (void)hipMemset(buf[0], 1, kBytes);
    (void)hipMemset(buf[1], 2, kBytes);
    (void)hipDeviceSynchronize();
    const dim3 grid(256 * 8), block(256);
    int launch = 0;
    auto rd = [&](auto wtag, int sparse) {
        constexpr int W = decltype(wtag)::value;
        const size_t n = kBytes / W;
        // alternate buffers so that no launch reads what the previous one wrote
        hipLaunchKernelGGL((k_read<W>), grid, block, 0, 0, (const typename Vec<W>::T*)buf[launch & 1], n, sparse,
                           sink);
        (void)hipDeviceSynchronize();
        printf("launch %2d read_w%d%s expected %.1f MiB\n", launch++, W, sparse ? "_44" : "",
               active_elems(n, sparse) * W / 1048576.0);
        // flush the Infinity Cache between launches: stream the other buffer
        (void)hipMemset(buf[launch & 1], 3, kBytes);
        (void)hipDeviceSynchronize();
    };
    auto wr = [&](auto wtag, int sparse) {
        constexpr int W = decltype(wtag)::value;
        const size_t n = kBytes / W;
        hipLaunchKernelGGL((k_write<W>), grid, block, 0, 0, (typename Vec<W>::T*)buf[launch & 1], n, sparse);
        (void)hipDeviceSynchronize();
        printf("launch %2d write_w%d%s expected %.1f MiB\n", launch++, W, sparse ? "_44" : "",
               active_elems(n, sparse) * W / 1048576.0);
        (void)hipMemset(buf[launch & 1], 3, kBytes);
        (void)hipDeviceSynchronize();
    };
    using I4 = std::integral_constant<int, 4>;
    using I8 = std::integral_constant<int, 8>;
    using I16 = std::integral_constant<int, 16>;
    for (int sparse = 0; sparse < 2; ++sparse) {
        rd(I4{}, sparse);
        rd(I8{}, sparse);
        rd(I16{}, sparse);
        wr(I4{}, sparse);
        wr(I8{}, sparse);
        wr(I16{}, sparse);
    }
    return 0;
}
