// ldpc5g_sparse.hip — decode_ldpc(LLRin, H, L, algo, alpha, beta) for an ARBITRARY binary
// parity-check matrix H (py5gphy/ldpc/nr_ldpc_decode.py:51-143), float64, all three algorithms:
//
//   min-sum family : _min_sum_process (:178-227) with its three zero-count branches restated as
//                    written (no zero: two smallest |Lq| of the row; one zero: only that edge gets
//                    alpha * prod(sign of the others) * max(min|others| - beta, 0); >= 2 zeros: 0),
//                    so any beta (negative included) gives the reference's messages;
//   BP             : _BP_process (:145-176): tanh products, clip to +-2*19.07, the one-zero edge
//                    gets the raw product of the others' tanh (no atanh), as the reference;
//   BF             : ldpc_decoder_BF (ldpc_decoder_bit_flipping.py:5-73).
//
// The 38.212 base graphs have their own specialised kernels (ldpc5g_dec*.hip); this one serves
// every other H the drop-in decode_ldpc is handed: it walks a CSR (rows: edges in ascending column
// order, as np.where(H[m,:]==1)) and a CSC (columns: entries in ascending row order, the order of
// Lr.sum(axis=0) at :126) built host-side from H.  One workgroup per codeblock; per-codeblock
// state (LQ per column, one double per edge) lives in LDS when it fits, else in a caller scratch.
// Flooding data flow as the reference: syndrome of LQ at the start of a pass (:107-114), every row
// from Lq = LQ_old - Lr_old (:129-131), LQ = LLR + row-ascending sum of Lr (:126), final
// LQ <= 0 decision + syndrome (:133-143).
#include <stdint.h>

#include "ldpc5g_common.h"

namespace ldpc5g_impl {
namespace {

constexpr int kSpThreads = 256;
constexpr size_t kSpLdsMax = 156 * 1024;   // of the CU's 160 KB (the BF kernel adds a static word)
constexpr double kBpClip = 2.0 * 19.07;   // nr_ldpc_decode.py:159,161

__device__ __noinline__ double sp_tanh_half(double q) { return tanh(q / 2); }
__device__ __noinline__ double sp_two_atanh(double x) { return 2.0 * atanh(x); }

// ------------------------------------------------------------------ min-sum family and BP
template <int ALGO, bool LDS>
__global__ __launch_bounds__(kSpThreads) void ldpc_sparse_soft_kernel(
    const double* __restrict__ llr, int64_t ldl, SparseH h, int8_t* __restrict__ ck, int64_t ldc,
    uint8_t* __restrict__ status, int32_t* __restrict__ iters, double* __restrict__ scratch, int L,
    double alpha, double beta) {
    extern __shared__ __align__(16) unsigned char smem[];
    const int cb = blockIdx.x;
    const double* lrow = llr + (int64_t)cb * ldl;
    int8_t* crow = ck + (int64_t)cb * ldc;
    double* LQ = LDS ? (double*)smem : scratch + (int64_t)cb * (h.N + h.E);
    double* Lr = LQ + h.N;   // per edge: Lr between passes; Lq (min-sum) / tanh(Lq/2) (BP) inside one
    const int t = threadIdx.x, nt = blockDim.x;
    for (int n = t; n < h.N; n += nt) LQ[n] = lrow[n];   // LQ = LLRin, Lq = H * LLRin (:94-98)
    for (int e = t; e < h.E; e += nt) Lr[e] = 0.0;       // (:101)
    __syncthreads();
    for (int it = 0; it < L; ++it) {
        bool fail = false;   // ck = LQ < 0; S = H ck mod 2 (:107-111)
        for (int m = t; m < h.M; m += nt) {
            int par = 0;
            for (int e = h.row_ptr[m]; e < h.row_ptr[m + 1]; ++e) par ^= LQ[h.col_idx[e]] < 0.0;
            fail |= par != 0;
        }
        if (!__syncthreads_or(fail)) {   // (:112-114)
            for (int n = t; n < h.N; n += nt) crow[n] = (int8_t)(LQ[n] < 0.0);
            if (t == 0) status[cb] = 1, iters[cb] = it;
            return;
        }
        for (int m = t; m < h.M; m += nt) {   // every row from the previous pass's LQ (:117-123)
            const int e0 = h.row_ptr[m], e1 = h.row_ptr[m + 1];
            if constexpr (ALGO == LDPC5G_ALGO_MS) {
                double min1 = __builtin_inf(), min2 = __builtin_inf();
                int s = 0, nz = 0;
                for (int e = e0; e < e1; ++e) {
                    const double q = LQ[h.col_idx[e]] - Lr[e];
                    Lr[e] = q;
                    const double a = fabs(q);
                    if (a < min1) min2 = min1, min1 = a;
                    else if (a < min2) min2 = a;   // a tie with min1 makes min2 == min1 (sorted[1])
                    s ^= q < 0.0;
                    nz += q == 0.0;
                }
                for (int e = e0; e < e1; ++e) {
                    const double q = Lr[e];
                    double r = 0.0;
                    if (nz == 0) {           // (:188-202)
                        const double mag = fabs(q) == min1 ? min2 : min1;
                        double v = mag - beta;
                        v = 0.0 > v ? 0.0 : v;   // Python max(v, 0)
                        r = alpha * v;
                        r = ((q < 0.0) != (s != 0)) ? -r : r;
                    } else if (nz == 1 && q == 0.0) {   // (:203-221): min / sign of the others
                        double v = min2 - beta;
                        v = 0.0 > v ? 0.0 : v;
                        r = alpha * v;
                        r = s ? -r : r;
                    }                        // other edges of a one-zero row, >= 2 zeros: 0 (:205, :224)
                    Lr[e] = r;
                }
            } else {   // BP
                double prod = 1.0, pa = 1.0, pb = 1.0;
                int nz = 0, zk = -1;
                for (int e = e0; e < e1; ++e) {
                    const double q = LQ[h.col_idx[e]] - Lr[e];
                    const double tq = sp_tanh_half(q);   // tanh(Lq/2) (:152, :165)
                    Lr[e] = tq;
                    prod = prod * tq;                   // np.prod, left to right (:154)
                    if (q == 0.0) {
                        if (nz == 0) zk = e;
                        ++nz;
                    } else if (nz == 0) {
                        pa = pa * tq;                   // prod(tanh_Lq[0:zero_idx])
                    } else {
                        pb = pb * tq;                   // prod(tanh_Lq[zero_idx+1:])
                    }
                }
                for (int e = e0; e < e1; ++e) {
                    double r = 0.0;
                    if (nz == 0) {
                        const double tmp2 = prod / Lr[e];
                        r = tmp2 >= 1.0 ? kBpClip : (tmp2 <= -1.0 ? -kBpClip : sp_two_atanh(tmp2));
                    } else if (nz == 1 && e == zk) {
                        r = pa * pb;                    // (:170): the product itself, no atanh
                    }
                    Lr[e] = r;
                }
            }
        }
        __syncthreads();
        for (int n = t; n < h.N; n += nt) {   // LQ = LLRin + Lr.sum(axis=0), rows ascending (:126)
            double acc = 0.0;
            for (int k = h.col_ptr[n]; k < h.col_ptr[n + 1]; ++k) acc = acc + Lr[h.col_edge[k]];
            LQ[n] = lrow[n] + acc;
        }
        __syncthreads();
    }
    // L passes without a zero syndrome: ck = LQ <= 0, status = final syndrome (:133-143)
    bool fail = false;
    for (int m = t; m < h.M; m += nt) {
        int par = 0;
        for (int e = h.row_ptr[m]; e < h.row_ptr[m + 1]; ++e) par ^= LQ[h.col_idx[e]] <= 0.0;
        fail |= par != 0;
    }
    fail = __syncthreads_or(fail);
    for (int n = t; n < h.N; n += nt) crow[n] = (int8_t)(LQ[n] <= 0.0);
    if (t == 0) status[cb] = !fail, iters[cb] = L;
}

// --------------------------------------------------------------------------------------- BF
template <bool LDS>
__global__ __launch_bounds__(kSpThreads) void ldpc_sparse_bf_kernel(
    const double* __restrict__ llr, int64_t ldl, SparseH h, int8_t* __restrict__ ck, int64_t ldc,
    uint8_t* __restrict__ status, int32_t* __restrict__ iters, unsigned char* __restrict__ scratch,
    int64_t stride, int L) {
    extern __shared__ __align__(16) unsigned char smem[];
    __shared__ int mx;
    const int cb = blockIdx.x;
    const double* lrow = llr + (int64_t)cb * ldl;
    int8_t* crow = ck + (int64_t)cb * ldc;
    unsigned char* base = LDS ? smem : scratch + (int64_t)cb * stride;
    int* En = (int*)base;                          // [N]
    int8_t* hd = (int8_t*)(En + h.N);              // [N]
    int8_t* S = hd + h.N;                          // [M]
    const int t = threadIdx.x, nt = blockDim.x;
    for (int n = t; n < h.N; n += nt) hd[n] = (int8_t)(lrow[n] < 0.0);   // LLR == 0 stays 0 (:41-43)
    for (int it = 0; it < L; ++it) {
        if (t == 0) mx = INT32_MIN;
        __syncthreads();
        bool fail = false;   // S = H ck mod 2 (:47)
        for (int m = t; m < h.M; m += nt) {
            int par = 0;
            for (int e = h.row_ptr[m]; e < h.row_ptr[m + 1]; ++e) par ^= hd[h.col_idx[e]];
            S[m] = (int8_t)par;
            fail |= par != 0;
        }
        if (!__syncthreads_or(fail)) {   // (:54-56)
            for (int n = t; n < h.N; n += nt) crow[n] = hd[n];
            if (t == 0) status[cb] = 1, iters[cb] = it;
            return;
        }
        int lmax = INT32_MIN;   // En = (2S - 1) @ H (:61), max (:67)
        for (int n = t; n < h.N; n += nt) {
            int acc = 0;
            for (int k = h.col_ptr[n]; k < h.col_ptr[n + 1]; ++k) acc += 2 * S[h.col_row[k]] - 1;
            En[n] = acc;
            lmax = acc > lmax ? acc : lmax;
        }
        atomicMax(&mx, lmax);
        __syncthreads();
        const int M = mx;
        for (int n = t; n < h.N; n += nt)
            if (En[n] == M) hd[n] ^= 1;   // flip every bit at the maximum (:70)
        __syncthreads();
    }
    for (int n = t; n < h.N; n += nt) crow[n] = hd[n];   // (ck, False) (:72-73)
    if (t == 0) status[cb] = 0, iters[cb] = L;
}

template <int ALGO>
int launch_soft(const double* llr, int64_t ldl, const SparseH& h, int8_t* ck, int64_t ldc,
                uint8_t* status, int32_t* iters, double* scratch, int B, int L, double alpha,
                double beta, hipStream_t st) {
    const size_t lds = sparse_lds_bytes(h.M, h.N, h.E, ALGO);
    if (lds) {
        if (int rc = set_lds_once<ldpc_sparse_soft_kernel<ALGO, true>>(kSpLdsMax)) return rc;
        hipLaunchKernelGGL((ldpc_sparse_soft_kernel<ALGO, true>), dim3(B), dim3(kSpThreads), lds, st,
                           llr, ldl, h, ck, ldc, status, iters, scratch, L, alpha, beta);
    } else {
        hipLaunchKernelGGL((ldpc_sparse_soft_kernel<ALGO, false>), dim3(B), dim3(kSpThreads), 0, st,
                           llr, ldl, h, ck, ldc, status, iters, scratch, L, alpha, beta);
    }
    return check_hip(hipGetLastError(), "ldpc_sparse_soft_kernel launch");
}

}  // namespace

// per-codeblock working set: soft (N + E) doubles; BF En int32 [N] + hd [N] + S [M] (16-B rounded)
int64_t sparse_cb_bytes(int M, int N, int E, int algo) {
    if (algo == LDPC5G_ALGO_BF) return (((int64_t)N * 5 + M + 15) / 16) * 16;
    return ((int64_t)N + E) * 8;
}

size_t sparse_lds_bytes(int M, int N, int E, int algo) {
    const int64_t b = sparse_cb_bytes(M, N, E, algo);
    return b <= (int64_t)kSpLdsMax ? (size_t)(b > 0 ? b : 16) : 0;
}

int launch_sparse(const double* llr, int64_t ldl, const SparseH& h, int8_t* ck, int64_t ldc,
                  uint8_t* status, int32_t* iters, void* scratch, int B, int L, int algo,
                  double alpha, double beta, hipStream_t st) {
    if (algo == LDPC5G_ALGO_MS)
        return launch_soft<LDPC5G_ALGO_MS>(llr, ldl, h, ck, ldc, status, iters, (double*)scratch, B, L,
                                           alpha, beta, st);
    if (algo == LDPC5G_ALGO_BP)
        return launch_soft<LDPC5G_ALGO_BP>(llr, ldl, h, ck, ldc, status, iters, (double*)scratch, B, L,
                                           alpha, beta, st);
    const size_t lds = sparse_lds_bytes(h.M, h.N, h.E, LDPC5G_ALGO_BF);
    if (lds) {
        if (int rc = set_lds_once<ldpc_sparse_bf_kernel<true>>(kSpLdsMax)) return rc;
        hipLaunchKernelGGL((ldpc_sparse_bf_kernel<true>), dim3(B), dim3(kSpThreads), lds, st, llr, ldl, h,
                           ck, ldc, status, iters, (unsigned char*)scratch, (int64_t)0, L);
    } else {
        hipLaunchKernelGGL((ldpc_sparse_bf_kernel<false>), dim3(B), dim3(kSpThreads), 0, st, llr, ldl, h,
                           ck, ldc, status, iters, (unsigned char*)scratch,
                           sparse_cb_bytes(h.M, h.N, h.E, LDPC5G_ALGO_BF), L);
    }
    return check_hip(hipGetLastError(), "ldpc_sparse_bf_kernel launch");
}

}  // namespace ldpc5g_impl
