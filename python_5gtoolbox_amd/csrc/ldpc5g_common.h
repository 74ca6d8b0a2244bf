// ldpc5g_common.h — shared device/host definitions of the MI355X 5G NR LDPC engine.
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include <atomic>
#include <type_traits>

#include "ldpc5g_tables.h"
#include "ldpc5g.h"

#define LDPC5G_VERSION "ldpc5g 0.2.0 gfx950"

namespace ldpc5g_impl {

// ------------------------------------------------------------------------------ base graphs
template <int BG>
struct BGT;
template <>
struct BGT<1> {
    static constexpr int MB = LDPC5G_BG1_ROWS;   // 46 base rows
    static constexpr int NB = LDPC5G_BG1_COLS;   // 68 base columns
    static constexpr int KB = 22;                // information columns
    static constexpr int KC = 26;                // core columns (degree > 1): info + 4 parity
    static constexpr int E = LDPC5G_BG1_EDGES;   // 316
    static constexpr const int16_t* RS = kBG1RowStart;
    static constexpr const int8_t* COL = kBG1Col;
};
template <>
struct BGT<2> {
    static constexpr int MB = LDPC5G_BG2_ROWS;   // 42
    static constexpr int NB = LDPC5G_BG2_COLS;   // 52
    static constexpr int KB = 10;
    static constexpr int KC = 14;
    static constexpr int E = LDPC5G_BG2_EDGES;   // 197
    static constexpr const int16_t* RS = kBG2RowStart;
    static constexpr const int8_t* COL = kBG2Col;
};

template <int BG>
constexpr int edge_of(int i, int j) {
    for (int e = BGT<BG>::RS[i]; e < BGT<BG>::RS[i + 1]; ++e)
        if (BGT<BG>::COL[e] == j) return e;
    return -1;
}

// V(i,j) mod Zc of edge e for lifting size index zi (tables packed 2 edges per 32-bit word so a
// wave-uniform read is a scalar load)
template <int BG>
__device__ __forceinline__ int shift_of(int zi, int e) {
    uint32_t w;
    if constexpr (BG == 1) w = kBG1ShiftMod[zi][e >> 1];
    else w = kBG2ShiftMod[zi][e >> 1];
    return (int)((e & 1) ? (w >> 16) : (w & 0xffffu));
}
template <int BG>
__device__ __forceinline__ int row_start_d(int i) {
    if constexpr (BG == 1) return kBG1RowStartD[i];
    else return kBG2RowStartD[i];
}
template <int BG>
__device__ __forceinline__ int col_d(int e) {
    if constexpr (BG == 1) return kBG1ColD[e];
    else return kBG2ColD[e];
}

// compile-time loop: f(std::integral_constant<int, I>) for I in [B, E)
template <int I, int E, typename F>
__device__ __forceinline__ void sfor(F&& f) {
    if constexpr (I < E) {
        f(std::integral_constant<int, I>{});
        sfor<I + 1, E>(f);
    }
}


// Workgroup barrier that orders LDS only.  __syncthreads() also releases global memory at
// workgroup scope, i.e. waits (vmcnt(0)) for every outstanding global load AND store of the wave;
// kernels that exchange data only through LDS use this one so stores and prefetches stay in flight.
__device__ __forceinline__ void lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

struct DecWork {     // one workgroup of the mixed-Zc path
    int32_t zi, Zc, G, first;
};
struct CbRef {       // one codeblock of the mixed-Zc path
    int64_t llr_off, ck_off;
    int32_t out, pad;
};

constexpr int kDecThreads = 384;   // = max Zc: one thread per check row z of a base row
constexpr int kCS = kDecThreads;   // LDS column stride (entries): G*Zc <= 384 always

// layered float32 kernel: 768-thread workgroups (12 waves = 3 per SIMD at <= 168 VGPRs) holding
// G = floor(768 / Zc) codeblocks, e.g. two BG1 Zc=384 codeblocks (384-thread workgroups, two per
// CU, measured 31 % slower: DESIGN.md §4.2)
constexpr int kDecThreadsL = 768;
inline int dec_threads(bool layered) { return layered ? kDecThreadsL : kDecThreads; }
inline int dec_G(int Zc, bool layered = false) {
    const int T = dec_threads(layered);
    return Zc >= T ? 1 : T / Zc;
}

// ---- host helpers (ldpc5g_capi.hip)
int fail(int code, const char* fmt, ...);
void clear_error();
const char* err_text();   // message of the last fail() on this thread
int zc_index(int Zc);
int check_hip(hipError_t e, const char* what);

// Raise kernel KERN's dynamic-LDS limit to `lds` bytes once per device: hipFuncSetAttribute is a
// host-side round trip that the per-codeblock drop-in calls would otherwise pay on every launch.
template <auto KERN>
int set_lds_once(size_t lds) {
    static std::atomic<uint64_t> done{0};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
    const uint64_t bit = 1ull << (dev & 63);
    if (done.load(std::memory_order_acquire) & bit) return 0;
    const hipError_t e = hipFuncSetAttribute((const void*)KERN, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return check_hip(e, "hipFuncSetAttribute");
    done.fetch_or(bit, std::memory_order_release);
    return 0;
}

// ---- launchers (one per translation unit)
int launch_encode(const int8_t* ck, int8_t* dn, int B, int bgn, int Zc, int zi, int64_t ldk,
                  int64_t ldn, hipStream_t st);
// workgroups of the decoder kernel resident per CU (HIP occupancy calculator), diagnostics
int dec_blocks_per_cu(int bgn, int dtype, bool layered);
// layered float32 instantiations (ldpc5g_dec_l.hip)
int dec_blocks_per_cu_l(int bgn);
int launch_dec_l(int bgn, const float* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B,
                 int Zc, int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
                 hipStream_t st);
// the dead-extension-row variants (LDPC5G_RATE_MATCHED): ldpc5g_dec_l_dead.hip / ldpc5g_dec_dead.hip
int launch_dec_l_dead(int bgn, const float* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B,
                      int Zc, int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta,
                      int pc, hipStream_t st);
int launch_dec_mixed_l_dead(int bgn, const float* llr, int8_t* ck, uint8_t* status, int32_t* iters,
                            int nwg, const DecWork* work, const CbRef* cbs, int L, double alpha,
                            double beta, int pc, hipStream_t st, bool zc384 = false);
int launch_flood_dead(int bgn, int dtype, const void* llr, int8_t* ck, uint8_t* status,
                      int32_t* iters, int B, int Zc, int zi, int64_t ldl, int64_t ldc, int L,
                      double alpha, double beta, int pc, hipStream_t st);
int launch_flood_mixed_dead(int bgn, int dtype, const void* llr, int8_t* ck, uint8_t* status,
                            int32_t* iters, int nwg, const DecWork* work, const CbRef* cbs, int L,
                            double alpha, double beta, int pc, hipStream_t st, bool zc384 = false);
int launch_flood_small(int bgn, int dtype, const void* llr, int8_t* ck, uint8_t* status, int32_t* iters,
                       int B, int Zc, int zi, int G, int64_t ldl, int64_t ldc, int L, double alpha,
                       double beta, int pc, hipStream_t st);
// float32 flooding instantiations, each in its own translation unit (parallel compiles)
int flood_blocks_per_cu_f32(int bgn);
int launch_flood_f32(int bgn, const float* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc,
                     int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc, hipStream_t st);
int launch_flood_mixed_f32(int bgn, const float* llr, int8_t* ck, uint8_t* status, int32_t* iters, int nwg,
                           const DecWork* work, const CbRef* cbs, int L, double alpha, double beta, int pc,
                           hipStream_t st);
int launch_flood_small_f32(int bgn, const float* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc,
                           int zi, int G, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
                           hipStream_t st);
int launch_flood_dead_f32(int bgn, const float* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B, int Zc,
                          int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
                          hipStream_t st);
int launch_flood_mixed_dead_f32(int bgn, const float* llr, int8_t* ck, uint8_t* status, int32_t* iters, int nwg,
                                const DecWork* work, const CbRef* cbs, int L, double alpha, double beta, int pc,
                                hipStream_t st);
int launch_dec_mixed_l(int bgn, const float* llr, int8_t* ck, uint8_t* status, int32_t* iters,
                       int nwg, const DecWork* work, const CbRef* cbs, int L, double alpha,
                       double beta, int pc, hipStream_t st, bool zc384 = false);
int launch_dec(int bgn, int dtype, bool layered, const void* llr, int8_t* ck, uint8_t* status,
               int32_t* iters, int B, int Zc, int zi, int64_t ldl, int64_t ldc, int L,
               double alpha, double beta, int pc, bool dead, hipStream_t st);
int launch_dec_mixed(int bgn, int dtype, bool layered, const void* llr, int8_t* ck,
                     uint8_t* status, int32_t* iters, int nwg, const DecWork* work,
                     const CbRef* cbs, int L, double alpha, double beta, int pc, bool dead,
                     hipStream_t st, bool zc384 = false);
// float64 flooding of a few large codeblocks, each over W = split_parts workgroups
// (ldpc5g_dec_split.hip); split_wanted: the chunks per wave R (1 or 2) of a launch it serves, or 0
int split_parts(int bgn, int Zc, int R);
int split_wanted(int bgn, int B, int Zc);
int launch_flood_split(int bgn, const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, int B,
                       int Zc, int zi, int64_t ldl, int64_t ldc, int L, double alpha, double beta,
                       int pc, hipStream_t st);
int split_timeouts(uint32_t* count);   // codeblocks whose split decode timed out (this device)
// float64 flooding of Zc = 384 batches: the frame kernel (ldpc5g_dec_frame.h), one translation unit
// per (base graph, DEAD) so they compile in parallel (ldpc5g_dec_frame{1,2}{,_dead}.hip)
constexpr int kFrameZc = 384;
template <int BG, bool DEAD>
int launch_frame_bg(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters, int nwg, int64_t ldl,
                    int64_t ldc, int L, double alpha, double beta, int pc, const DecWork* work,
                    const CbRef* cbs, hipStream_t st);
inline int launch_frame(int bgn, bool dead, const double* llr, int8_t* ck, uint8_t* status, int32_t* iters,
                        int nwg, int64_t ldl, int64_t ldc, int L, double alpha, double beta, int pc,
                        const DecWork* work, const CbRef* cbs, hipStream_t st) {
    if (bgn == 1)
        return dead ? launch_frame_bg<1, true>(llr, ck, status, iters, nwg, ldl, ldc, L, alpha, beta, pc, work, cbs, st)
                    : launch_frame_bg<1, false>(llr, ck, status, iters, nwg, ldl, ldc, L, alpha, beta, pc, work, cbs, st);
    return dead ? launch_frame_bg<2, true>(llr, ck, status, iters, nwg, ldl, ldc, L, alpha, beta, pc, work, cbs, st)
                : launch_frame_bg<2, false>(llr, ck, status, iters, nwg, ldl, ldc, L, alpha, beta, pc, work, cbs, st);
}
int launch_bf(int bgn, int dtype, const void* llr, int8_t* ck, uint8_t* status, int32_t* iters,
              int B, int Zc, int zi, int64_t ldl, int64_t ldc, int L, int pc, hipStream_t st);
int launch_bp(int bgn, const double* llr, int8_t* ck, uint8_t* status, int32_t* iters,
              double* msg, int B, int Zc, int zi, int64_t ldl, int64_t ldc, int L, int pc,
              hipStream_t st);
int edges_of_bg(int bgn);
// BP message scratch per codeblock, in units of Zc doubles (2 x the row-edge pair slots)
int bp_scratch_per_zc(int bgn);

// ---- arbitrary parity-check matrices (ldpc5g_sparse.hip): CSR rows (edges in ascending column
// order) + CSC columns (entries in ascending row order: edge id and row)
struct SparseH {
    const int32_t* row_ptr;    // [M + 1]
    const int32_t* col_idx;    // [E] column of edge e (edges numbered row-major)
    const int32_t* col_ptr;    // [N + 1]
    const int32_t* col_edge;   // [E] edge ids of column n, rows ascending
    const int32_t* col_row;    // [E] their rows
    int32_t M, N, E, pad;
};
int64_t sparse_cb_bytes(int M, int N, int E, int algo);
size_t sparse_lds_bytes(int M, int N, int E, int algo);   // 0: the working set needs the scratch
int launch_sparse(const double* llr, int64_t ldl, const SparseH& h, int8_t* ck, int64_t ldc,
                  uint8_t* status, int32_t* iters, void* scratch, int B, int L, int algo,
                  double alpha, double beta, hipStream_t st);

// Host -> device copy of a small host-built plan on `st` through a per-thread ring of pinned
// staging buffers: returns once the copy is queued; a slot is reused only after the event
// recorded behind its previous copy has completed (ldpc5g_capi.hip).
int stage_h2d(void* dst, const void* src, size_t n, hipStream_t st);

}  // namespace ldpc5g_impl
