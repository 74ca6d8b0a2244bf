// FETCH_SIZE / WRITE_SIZE calibration (MI355X_MICROARCH.md §HBM: "other access widths are
// uncalibrated: calibrate on a known byte count in your own access pattern").  Streams a 1 GiB
// buffer (4x the Infinity Cache) with coalesced W-byte-per-lane loads (W = 4, 8, 16: the
// decoders read float32 / float64 LLRs, the encoder 16-B pieces) and writes one with W-byte
// stores; each kernel is launched once with a known byte count.  Run under
//   rocprofv3 --pmc FETCH_SIZE -- ./fetch_calib   and   rocprofv3 --pmc WRITE_SIZE -- ./fetch_calib
// and divide the counter (KiB) by the bytes printed here (tools/microbench/fetch_calib.py).
#include <hip/hip_runtime.h>
#include <stdio.h>

template <typename V>
__global__ __launch_bounds__(256) void rd_kernel(const V* __restrict__ p, size_t n, float* out) {
    float acc = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
        const V v = p[i];
        acc += __builtin_bit_cast(float, ((const unsigned*)&v)[0]);
    }
    if (acc == 1.2345f) out[0] = acc;   // keep the loads; never true for the zero-filled buffer
}
template <typename V>
__global__ __launch_bounds__(256) void wr_kernel(V* __restrict__ p, size_t n) {
    V z{};
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = z;
}
struct alignas(8) B8 { unsigned a, b; };
struct alignas(16) B16 { unsigned a, b, c, d; };

int main() {
    const size_t bytes = 1ull << 30;
    void* buf = nullptr;
    float* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(buf, 0, bytes);
    const dim3 grid(256 * 16);
    hipLaunchKernelGGL(rd_kernel<unsigned>, grid, dim3(256), 0, 0, (const unsigned*)buf, bytes / 4, out);
    hipLaunchKernelGGL(rd_kernel<B8>, grid, dim3(256), 0, 0, (const B8*)buf, bytes / 8, out);
    hipLaunchKernelGGL(rd_kernel<B16>, grid, dim3(256), 0, 0, (const B16*)buf, bytes / 16, out);
    hipLaunchKernelGGL(wr_kernel<unsigned>, grid, dim3(256), 0, 0, (unsigned*)buf, bytes / 4);
    hipLaunchKernelGGL(wr_kernel<B8>, grid, dim3(256), 0, 0, (B8*)buf, bytes / 8);
    hipLaunchKernelGGL(wr_kernel<B16>, grid, dim3(256), 0, 0, (B16*)buf, bytes / 16);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    printf("{\"bytes_per_kernel\": %zu}\n", bytes);
    return 0;
}
