// Co-residency probe (dev tool): do two 384-thread workgroups with a given VGPR/LDS footprint
// share a CU?  Each workgroup spins ~50 us and records (smid, start, end).
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>
#include <map>
template <int WPE>
__global__ __launch_bounds__(384) __attribute__((amdgpu_waves_per_eu(WPE))) void spin(unsigned long long* rec, int iters) {
    extern __shared__ int sm[];
    unsigned long long t0 = wall_clock64();
    float a = threadIdx.x;
    for (int i = 0; i < iters; ++i) { a = a * 1.0001f + 0.5f; }
    sm[threadIdx.x] = (int)a;
    __syncthreads();
    unsigned long long t1 = wall_clock64();
    if (threadIdx.x == 0) {
        rec[blockIdx.x * 3 + 0] = __smid();
        rec[blockIdx.x * 3 + 1] = t0;
        rec[blockIdx.x * 3 + 2] = t1 + sm[5] * 0;
    }
}
template <int WPE>
void run(int lds_kb, int nblk) {
    unsigned long long* d; hipMalloc(&d, nblk * 3 * 8);
    size_t lds = lds_kb * 1024;
    hipFuncSetAttribute((const void*)spin<WPE>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    int occ = -1; hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spin<WPE>, 384, lds);
    spin<WPE><<<nblk, 384, lds>>>(d, 200000);
    hipDeviceSynchronize();
    std::vector<unsigned long long> h(nblk * 3);
    hipMemcpy(h.data(), d, nblk * 3 * 8, hipMemcpyDeviceToHost);
    std::map<unsigned long long, std::vector<std::pair<unsigned long long, unsigned long long>>> byCU;
    for (int b = 0; b < nblk; ++b) byCU[h[b * 3]].push_back({h[b * 3 + 1], h[b * 3 + 2]});
    int overl = 0, pairs = 0;
    for (auto& kv : byCU) {
        auto& v = kv.second;
        for (size_t i = 0; i < v.size(); ++i) for (size_t j = i + 1; j < v.size(); ++j) {
            ++pairs;
            if (v[i].first < v[j].second && v[j].first < v[i].second) ++overl;
        }
    }
    printf("WPE=%d LDS=%d KB blocks=%d: occupancy calc %d/CU, distinct smid %zu, same-CU pairs %d, overlapping %d\n",
           WPE, lds_kb, nblk, occ, byCU.size(), pairs, overl);
    hipFree(d);
}
int main() {
    for (int kb : {8, 43, 77}) { run<3>(kb, 512); run<1>(kb, 512); }
    return 0;
}
