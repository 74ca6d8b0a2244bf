/*
 * ldpc5g.h — C ABI of the MI355X-native 5G NR LDPC engine (libldpc5g.so, gfx950).
 *
 * The engine replaces the hot path of the reference py5gphy/ldpc package:
 *   ldpc5g_encode        <- py5gphy/ldpc/nr_ldpc_encode.py:8     encode_ldpc(ck, bgn)
 *                           (+ _gen_ldpc_parity_bit :52-115), batched over codeblocks
 *   ldpc5g_decode_ms     <- py5gphy/ldpc/nr_ldpc_decode.py:11    nr_decode_ldpc(LLRin, Zc, bgn, L,
 *                           'min-sum', alpha, beta) and decode_ldpc :51-143 / _min_sum_process
 *                           :178-227, batched over codeblocks
 *   ldpc5g_decode_ms_mixed  the same over a batch of codeblocks with per-codeblock (bgn, Zc),
 *                           the shape DLSCHDecode (py5gphy/nr_pdsch/nr_dlsch_decode.py:62-91)
 *                           and ULSCH_decoding (py5gphy/nr_pusch/nr_ulsch_decode.py:92) feed
 *   ldpc5g_find_ils      <- py5gphy/ldpc/ldpc_info.py:81         find_iLS(Zc)
 *
 * Conventions
 *   - All buffer pointers are DEVICE pointers (hipMalloc / torch tensors); the library never
 *     allocates or frees caller buffers.  `stream` is a hipStream_t (NULL = default stream).
 *   - Bits are int8 per bit (0/1, -1 = filler), LLRs are log(P0/P1) (positive => bit 0).
 *   - Calls are asynchronous on `stream` and reentrant; ldpc5g_last_error() is thread-local.
 *   - Return 0 on success, or a negative code: the Python host maps them to AssertionError,
 *     as the reference's `assert` checks (nr_ldpc_encode.py:18,29; nr_ldpc_decode.py:23-37).
 */
#ifndef LDPC5G_H
#define LDPC5G_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LDPC5G_OK 0
#define LDPC5G_EBGN (-1)   /* bgn not in {1,2}                                 */
#define LDPC5G_EZC (-2)    /* Zc not a TS 38.212 lifting size (find_iLS == 255) */
#define LDPC5G_ESIZE (-3)  /* bad batch / stride / L / dtype / schedule        */
#define LDPC5G_EHIP (-4)   /* HIP runtime error (launch failure)               */

/* LLR element types */
#define LDPC5G_F64 0       /* float64: bit-exact with the reference's numpy float64 decoder */
#define LDPC5G_F32 1       /* float32 */

/* decode flags */
#define LDPC5G_LLR_FULL 1  /* LLR rows hold all Nf = 68Zc/52Zc columns, the 2Zc punctured ones
                              included (decode_ldpc(LLRin, H, ...) input, nr_ldpc_decode.py:51) */
#define LDPC5G_RATE_MATCHED 2  /* LLR rows come from rate recovery (nr_ldpc_raterecover.py:6-65):
                              extension columns that were never transmitted hold +0.0.  The
                              decoder detects rows whose extension column is +0.0 in every
                              codeblock of a workgroup and skips their (provably null) updates;
                              results are bit-identical to the plain decode.  Ignored by launches
                              of <= 64 codeblock slots (one small codeblock) and by BF / BP. */

/* decoding schedules */
#define LDPC5G_FLOODING 0  /* the reference's two-phase (Jacobi) schedule, nr_ldpc_decode.py:105-131 */
#define LDPC5G_LAYERED 1   /* row-block serial schedule (perf mode, float32 only)                  */

/* Lifting-set index 0..7 of Zc (TS 38.212 Table 5.3.2-1), 255 if Zc is not a lifting size. */
int ldpc5g_find_ils(int32_t Zc);

/* Encode B codeblocks.
 *   ck : [B][ldk] int8, first K = 22*Zc (bgn 1) / 10*Zc (bgn 2) entries used, values 0/1/-1
 *   dn : [B][ldn] int8, first N = 66*Zc / 50*Zc entries written:
 *        dn[0:K-2Zc] = ck[2Zc:K] (fillers stay -1), dn[K-2Zc:N] = parity bits.
 *   Parity treats ck[k] = -1 (k >= 2Zc) as 0, exactly as the reference zeroes fillers before
 *   encoding.  ck is not modified (the reference's in-place filler zeroing is done host-side). */
int ldpc5g_encode(const int8_t* ck, int8_t* dn, int32_t B, int32_t bgn, int32_t Zc,
                  int64_t ldk, int64_t ldn, void* stream);

/* Min-sum decode (MS / normalized alpha<1 / offset beta>0 / mixed) of B codeblocks.
 *   llr    : [B][ldl] of llr_dtype, N = 66*Zc / 50*Zc entries (2*Zc systematic bits punctured,
 *            decoded with LLR 0), or Nf = 68*Zc / 52*Zc entries when flags & LDPC5G_LLR_FULL
 *   ck     : [B][ldc] int8, Nf = 68*Zc / 52*Zc hard decisions written (blkandcrc = ck[0:K])
 *   status : [B] uint8, 1 iff ck satisfies every parity check
 *   iters  : [B] int32, check-node updates performed (flooding: the reference's loop index at
 *            its early return, else L; layered: iterations run)
 *   schedule LDPC5G_FLOODING works with F64 (bit-exact with the reference) and F32;
 *   LDPC5G_LAYERED requires F32.
 *   The codeblocks sharing a workgroup (up to 768 / Zc of them) are addressed with 32-bit byte
 *   offsets: G * ldl * sizeof(element) >= 4 GiB returns LDPC5G_ESIZE (an ldl of 2^26 or more). */
int ldpc5g_decode_ms(const void* llr, int32_t llr_dtype, int8_t* ck, uint8_t* status,
                     int32_t* iters, int32_t B, int32_t bgn, int32_t Zc, int32_t L,
                     double alpha, double beta, int32_t schedule, int32_t flags, int64_t ldl,
                     int64_t ldc, void* stream);

/* Per-codeblock drop-in shape, HOST buffers in and out  <- py5gphy/ldpc/nr_ldpc_decode.py:11-49
 * nr_decode_ldpc(LLRin, Zc, bgn, L, 'min-sum', alpha, beta) and nr_ldpc_encode.py:8 encode_ldpc(ck,
 * bgn), called one codeblock at a time by the reference's callers (nr_dlsch_decode.py:91,
 * scripts/internal/sim_ldpc_internal.py:50-58).  float64 flooding min-sum (bit-exact with the
 * reference) / the encoder on B contiguous host rows (llr [B][N or Nf], ck [B][Nf], status [B],
 * iters [B]; ck [B][K], dn [B][N]): the rows go through a pinned staging buffer and a device
 * buffer kept per thread AND per device ordinal (< 64; grown on demand and held for the life of
 * the process, so a thread that alternates devices reuses each device's pair), one H2D copy,
 * the kernel, one D2H copy and one synchronisation of `stream` — no caller-side device memory.
 * Synchronous: returns when the outputs are written.  beta < 0 is rejected (see decode_sparse). */
int ldpc5g_decode_ms_host(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters,
                          int32_t B, int32_t bgn, int32_t Zc, int32_t L, double alpha, double beta,
                          int32_t flags, void* stream);
int ldpc5g_encode_host(const int8_t* ck, int8_t* dn, int32_t B, int32_t bgn, int32_t Zc,
                       void* stream);

/* Hard-decision bit flipping (algo='BF')  <- py5gphy/ldpc/ldpc_decoder_bit_flipping.py:5-73
 * reached through nr_decode_ldpc(..., algo='BF') (nr_ldpc_decode.py:65-67).  Same buffers as
 * ldpc5g_decode_ms; ck holds the 0/1 decisions (the reference returns them as float64), status
 * is 0 after L iterations without a zero syndrome (the reference checks only at loop start). */
int ldpc5g_decode_bf(const void* llr, int32_t llr_dtype, int8_t* ck, uint8_t* status,
                     int32_t* iters, int32_t B, int32_t bgn, int32_t Zc, int32_t L,
                     int32_t flags, int64_t ldl, int64_t ldc, void* stream);

/* Float64 sum-product, flooding (algo='BP')  <- nr_ldpc_decode.py:51-143 + _BP_process :145-176.
 * Per-edge messages do not compress: the caller provides a float64 device scratch of
 * ldpc5g_bp_scratch_elems(B, bgn, Zc) elements (-1 on bad arguments). */
int64_t ldpc5g_bp_scratch_elems(int32_t B, int32_t bgn, int32_t Zc);
int ldpc5g_decode_bp(const double* llr, int8_t* ck, uint8_t* status, int32_t* iters,
                     double* scratch, int64_t scratch_elems, int32_t B, int32_t bgn, int32_t Zc,
                     int32_t L, int32_t flags, int64_t ldl, int64_t ldc, void* stream);

/* ---- arbitrary parity-check matrix  <- py5gphy/ldpc/nr_ldpc_decode.py:51-143 decode_ldpc(LLRin, H,
 * L, algo, alpha, beta) for ANY binary H (the 38.212 expansions have the specialised entry points
 * above).  H is passed as a CSR of its rows plus a CSC of its columns (DEVICE int32 arrays):
 *   row_ptr [M+1], col_idx [E]   edges of row m = col_idx[row_ptr[m] .. row_ptr[m+1]), columns
 *                                ascending (np.where(H[m,:] == 1), :80-83); edges numbered row-major
 *   col_ptr [N+1], col_edge [E], col_row [E]   entries of column n, rows ascending (np.where(
 *                                H[:,n] == 1), :88-91): the edge id and its row
 * algo LDPC5G_ALGO_MS: the min-sum family with the reference's zero-count branches (:178-227), any
 * beta; LDPC5G_ALGO_BP: sum-product (:145-176); LDPC5G_ALGO_BF: bit flipping
 * (ldpc_decoder_bit_flipping.py:5-73).  All float64, flooding, B codeblocks of N LLRs each:
 *   llr [B][ldl] float64, ck [B][ldc] int8 (N decisions), status [B] uint8, iters [B] int32.
 * A min-sum row of degree < 2 makes the reference raise (np.sort(...)[1]) once a check-node update
 * runs; the kernel computes on, and the Python host raises the reference's error from iters/status.
 * Per-codeblock state lives in LDS when it fits (ldpc5g_sparse_scratch_bytes returns 0), else in
 * a caller DEVICE scratch of ldpc5g_sparse_scratch_bytes(B, M, N, E, algo) bytes (-1: bad args). */
#define LDPC5G_ALGO_MS 0
#define LDPC5G_ALGO_BP 1
#define LDPC5G_ALGO_BF 2
int64_t ldpc5g_sparse_scratch_bytes(int32_t B, int32_t M, int32_t N, int32_t E, int32_t algo);
int ldpc5g_decode_sparse(const double* llr, int64_t ldl, int32_t B, int32_t M, int32_t N, int32_t E,
                         const int32_t* row_ptr, const int32_t* col_idx, const int32_t* col_ptr,
                         const int32_t* col_edge, const int32_t* col_row, int32_t L, int32_t algo,
                         double alpha, double beta, int8_t* ck, int64_t ldc, uint8_t* status,
                         int32_t* iters, void* scratch, int64_t scratch_bytes, void* stream);

/* One codeblock of a mixed batch: base graph, lifting size, element offsets of its LLR row
 * (into llr_base, in elements) and of its ck row (into ck_base, in bytes). */
typedef struct {
    int32_t bgn;
    int32_t Zc;
    int64_t llr_off;
    int64_t ck_off;
} ldpc5g_cb_desc_t;

/* Decode a batch of codeblocks with heterogeneous (bgn, Zc) in at most two launches (one per
 * base graph).  `desc` is a HOST array of B descriptors; status[b] / iters[b] follow desc order.
 * The work list is built on the host and copied into a stream-ordered allocation
 * (hipMallocAsync / hipFreeAsync on `stream`) from a per-thread pool of pinned staging buffers:
 * the call returns once the copy is queued.  The pool grows with the plans in flight (a slot is
 * reused once its copy has completed) up to 64 slots per thread, and only past 64 plans in flight
 * does a call wait for the oldest copy.  The pool's pinned memory is held by each calling thread
 * for the life of the process (about the size of its largest plans).  Repeated decodes of one batch shape should build the
 * plan once instead (ldpc5g_mixed_plan + ldpc5g_decode_ms_mixed_plan). */
int ldpc5g_decode_ms_mixed(const ldpc5g_cb_desc_t* desc, int32_t B, const void* llr_base,
                           int32_t llr_dtype, int8_t* ck_base, uint8_t* status, int32_t* iters,
                           int32_t L, double alpha, double beta, int32_t schedule,
                           int32_t flags, void* stream);

/* Build the work list (plan) of a mixed batch into the caller's HOST buffer `plan` (pinned memory
 * recommended, `plan_bytes` long).  Returns the plan size in bytes (>= 0; the buffer is untouched
 * when it is too small, so a first call with plan_bytes = 0 sizes it) or a negative error.  The
 * plan depends only on (desc, B, schedule).  Layout (opaque to callers): a 32-byte header, the
 * workgroups of each base graph by lifting size (BG1 Zc = 384 last, a partly filled workgroup
 * before the full ones), the codeblock references (sorted by llr_off within a workgroup: the
 * kernels address a workgroup's rows from its lowest one with 32-bit offsets, so the rows of the
 * codeblocks packed together — same (bgn, Zc), consecutive in desc order — must span < 4 GiB,
 * else LDPC5G_ESIZE). */
int64_t ldpc5g_mixed_plan(const ldpc5g_cb_desc_t* desc, int32_t B, int32_t schedule, void* plan,
                          int64_t plan_bytes);

/* Decode with a plan the caller copied to the device (`plan_dev`, the bytes ldpc5g_mixed_plan
 * wrote, on this stream's device): <= 2 launches, nothing else — no allocation, no copy, no
 * synchronisation.  schedule must be the one the plan was built for. */
int ldpc5g_decode_ms_mixed_plan(const void* plan_dev, const void* plan_host, const void* llr_base,
                                int32_t llr_dtype, int8_t* ck_base, uint8_t* status,
                                int32_t* iters, int32_t L, double alpha, double beta,
                                int32_t schedule, int32_t flags, void* stream);

/* ============================================================ DL-SCH / UL-SCH transport chain
 * TS 38.212 §7.2 (DL-SCH) / §6.2 (UL-SCH) around the codec, batched over T transport blocks that
 * share one configuration.  Bits are int8 0/1 (fillers -1); CRC remainders are uint32 with the
 * first CRC bit in bit L-1.  */

/* CRC generator ids (py5gphy/crc/crc.py:94-106) */
#define LDPC5G_CRC6 0
#define LDPC5G_CRC11 1
#define LDPC5G_CRC16 2
#define LDPC5G_CRC24A 3
#define LDPC5G_CRC24B 4
#define LDPC5G_CRC24C 5

/* CRC of `rows` bit rows ([rows][ld] int8, nbits each): rem[r] = M(x) x^L mod g(x), the parity
 * nr_crc_encode appends (crc.py:4-41, mask 0, bit L-1 first); a row that ends in its own CRC gives
 * 0 iff nr_crc_decode reports no error (crc.py:43-88).  rem must not alias bits. */
int ldpc5g_crc(const int8_t* bits, int64_t ld, int64_t nbits, int32_t rows, int32_t poly,
               uint32_t* rem, void* stream);

/* Shared-configuration geometry of a transport block (host struct, filled by ldpc5g_sch_config). */
typedef struct {
    int32_t A;            /* TBSize                                                           */
    int32_t B;            /* A + TB CRC length                                                */
    int32_t tb_crc_poly;  /* LDPC5G_CRC24A (A > 3824) or LDPC5G_CRC16 (nr_dlsch.py:34-40)      */
    int32_t bgn;          /* base graph (nr_dlsch.py:44-49)                                   */
    int32_t C, cbz, Lcb, F, K, K_apo, Zc;   /* get_cbs_info (ldpc_info.py:5-78); K_apo = cbz+Lcb */
    int32_t N, Ncb, k0;   /* codeword length, circular buffer (Nref / N), rv start             */
    int32_t Qm, NL, rv;
    int32_t E_lo, E_hi, c_switch;   /* Er: codeblocks c < c_switch get E_lo, the others E_hi    */
    int64_t G;            /* the G that sized Er (nr_ldpc_ratematch.py:5-27)                   */
    int64_t E_total;      /* sum of Er = bits of g per transport block                         */
} ldpc5g_sch_cfg_t;

/* Fill cfg for a transport block: TBSize A, modulation order Qm, code rate * 1024, layers NL,
 * redundancy version rv, TBS_LBRM (> 0: DL-SCH limited buffer Nref = floor(TBS_LBRM / (2C/3)),
 * nr_dlsch.py:63-65; 0: UL-SCH Ncb = N, nr_ulsch.py:55-58) and G (rate-matching output bits).
 * Float arithmetic of the reference (base-graph thresholds, k0, Er) is reproduced in double. */
int ldpc5g_sch_config(int32_t A, int32_t Qm, double coderateby1024, int32_t NL, int32_t rv,
                      int64_t TBS_LBRM, int64_t G, ldpc5g_sch_cfg_t* cfg);

/* DLSCHEncode (py5gphy/nr_pdsch/nr_dlsch.py:12-74) / ULSCH_Crc_CodeBlockSegment +
 * ULSCH_encoding_ratematch (nr_pusch/nr_ulsch.py:13-70) of T transport blocks:
 *   trblk [T][lda] int8 -> g [T][ldg] int8 (E_total bits each).
 * Workspaces (device, caller-owned): ck [T*C][K] int8 (codeblocks with CRC24B and -1 fillers,
 * as ldpc_cbsegment returns them), dn [T*C][N] int8 (encoder output), tb_crc [T] uint32 (the
 * TB CRC, also an output). */
int ldpc5g_sch_encode(const int8_t* trblk, int64_t lda, int8_t* g, int64_t ldg,
                      const ldpc5g_sch_cfg_t* cfg, int32_t T, int8_t* ck, int8_t* dn,
                      uint32_t* tb_crc, void* stream);

/* The two halves of ldpc5g_sch_encode:
 *   ldpc5g_sch_segment   TB CRC + codeblock segmentation + CRC24B (nr_dlsch.py:32-56,
 *                        ULSCH_Crc_CodeBlockSegment nr_ulsch.py:13-35): trblk -> ck, tb_crc
 *   ldpc5g_sch_ratematch LDPC encode + rate matching + concatenation (nr_dlsch.py:58-74,
 *                        ULSCH_encoding_ratematch nr_ulsch.py:37-70): ck -> dn -> g
 * ldpc5g_sch_ratematch reads only the codeblock fields of cfg (bgn, C, cbz, Lcb, K, K_apo, Zc,
 * N, Ncb, k0, Qm, E_lo, E_hi, c_switch). */
int ldpc5g_sch_segment(const int8_t* trblk, int64_t lda, const ldpc5g_sch_cfg_t* cfg, int32_t T,
                       int8_t* ck, uint32_t* tb_crc, void* stream);
int ldpc5g_sch_ratematch(const int8_t* ck, const ldpc5g_sch_cfg_t* cfg, int32_t T, int8_t* dn,
                         int8_t* g, int64_t ldg, void* stream);

/* Rate recovery (nr_ldpc_raterecover.py:6-65) of every codeblock + optional HARQ combining with
 * the previous decoder inputs (nr_dlsch_decode.py:73-88):
 *   llr [T][ldg] (llr_dtype) -> llr_dn [T*C][N] (dn_dtype); harq_in NULL or [T*C][N] dn_dtype,
 *   either disjoint from llr_dn or llr_dn itself (in-place combining with the previous call's
 *   output); a partial overlap is not supported.  (Every rate-recovery entry point below too.)
 * Computed in float64 like the reference (a float32 llr_dn is the float64 result rounded once). */
int ldpc5g_sch_raterecover(const void* llr, int32_t llr_dtype, int64_t ldg,
                           const ldpc5g_sch_cfg_t* cfg, int32_t T, const void* harq_in,
                           void* llr_dn, int32_t dn_dtype, void* stream);

/* TB reassembly and CRC checks (nr_dlsch_decode.py:93-106): ck [T*C][ldc] int8 hard decisions
 * -> tbblk [T][ldb] int8 (B = A + CRC bits: the TB and its CRC), cb_crc_ok [T*C] (CRC24B when
 * C > 1, else 1), tb_ok [T] (TB CRC), tb_rem [T] uint32 (TB CRC remainder, scratch + output). */
int ldpc5g_sch_tb_check(const int8_t* ck, int64_t ldc, const ldpc5g_sch_cfg_t* cfg, int32_t T,
                        int8_t* tbblk, int64_t ldb, uint8_t* cb_crc_ok, uint32_t* tb_rem,
                        uint8_t* tb_ok, void* stream);

/* DLSCHDecode (nr_dlsch_decode.py:13-110) / ULSCH_decoding (nr_ulsch_decode.py:13-110) with the
 * min-sum decoder: ldpc5g_sch_raterecover -> ldpc5g_decode_ms over the T*C codeblocks (ck
 * [T*C][Nf], status / iters [T*C]) -> ldpc5g_sch_tb_check.  Asynchronous on `stream`. */
int ldpc5g_sch_decode(const void* llr, int32_t llr_dtype, int64_t ldg, const ldpc5g_sch_cfg_t* cfg,
                      int32_t T, const void* harq_in, void* llr_dn, int32_t dn_dtype, int8_t* ck,
                      uint8_t* status, int32_t* iters, int32_t L, double alpha, double beta,
                      int32_t schedule, int8_t* tbblk, int64_t ldb, uint8_t* cb_crc_ok,
                      uint32_t* tb_rem, uint8_t* tb_ok, void* stream);

/* ---- transport blocks with per-TB configurations (the reference configures every TB of a slot
 * independently: nr_pdsch.py:212-281 -> DLSCHDecode at :281, nr_dlsch.py:12-74 per TB).
 * cfgs[T] (host, each from ldpc5g_sch_config); TB t's codeblocks occupy consecutive rows of the
 * flat workspaces, TB after TB: ck rows of K_t, dn / llr_dn rows of N_t, decoder ck rows of
 * Nf_t = 68/52 Zc_t, status / iters / cb_crc_ok one entry per codeblock.  trblk [T][lda] (A_t
 * bits used), g / llr [T][ldg] (E_total_t used), tbblk [T][ldb] (B_t used).
 * sizes[7] = {ck elements, dn elements, decoder-ck elements, codeblocks, max A, max B, max E}.
 * The per-TB geometry goes to the device like the mixed-Zc work list (stream-ordered allocation,
 * pinned staging pool: see ldpc5g_decode_ms_mixed). */
int ldpc5g_sch_multi_sizes(const ldpc5g_sch_cfg_t* cfgs, int32_t T, int64_t* sizes);
int ldpc5g_sch_encode_multi(const int8_t* trblk, int64_t lda, int8_t* g, int64_t ldg,
                            const ldpc5g_sch_cfg_t* cfgs, int32_t T, int8_t* ck, int8_t* dn,
                            uint32_t* tb_crc, void* stream);
/* rate recovery alone (raterecover_ldpc, py5gphy/ldpc/nr_ldpc_raterecover.py:6-65, + HARQ) of every
 * codeblock of the T transport blocks in ONE launch, into the flat llr_dn rows (N_t per codeblock,
 * TB after TB): the input of a mixed-Zc decode (ldpc5g_decode_ms_mixed_plan). */
int ldpc5g_sch_raterecover_multi(const void* llr, int32_t llr_dtype, int64_t ldg,
                                 const ldpc5g_sch_cfg_t* cfgs, int32_t T, const void* harq_in,
                                 void* llr_dn, int32_t dn_dtype, void* stream);
/* The same with the geometry built once: ldpc5g_sch_multi_plan writes the plan's host bytes (returns
 * the size needed; call with plan = NULL first), the caller copies them to device memory once, and
 * every ldpc5g_sch_raterecover_multi_plan(plan_dev, plan_host, ...) only launches (no host-side
 * validation, allocation or copy per call; asynchronous on `stream`). */
int64_t ldpc5g_sch_multi_plan(const ldpc5g_sch_cfg_t* cfgs, int32_t T, void* plan, int64_t plan_bytes);
int ldpc5g_sch_raterecover_multi_plan(const void* plan_dev, const void* plan_host, const void* llr,
                                      int32_t llr_dtype, int64_t ldg, const void* harq_in, void* llr_dn,
                                      int32_t dn_dtype, void* stream);
/* decode: rate recovery (+ HARQ, harq_in laid out like llr_dn) -> mixed-Zc min-sum decode of all
 * codeblocks (ldpc5g_decode_ms_mixed) -> TB reassembly + CRCs.  Asynchronous on `stream`. */
int ldpc5g_sch_decode_multi(const void* llr, int32_t llr_dtype, int64_t ldg,
                            const ldpc5g_sch_cfg_t* cfgs, int32_t T, const void* harq_in,
                            void* llr_dn, int32_t dn_dtype, int8_t* ck, uint8_t* status,
                            int32_t* iters, int32_t L, double alpha, double beta, int32_t schedule,
                            int8_t* tbblk, int64_t ldb, uint8_t* cb_crc_ok, uint32_t* tb_rem,
                            uint8_t* tb_ok, void* stream);

/* ================================================ scrambling, modulation, soft demodulation
 * The symbol-level steps either side of the DL-SCH chain (TS 38.211 5.2.1, 5.1, 7.3.1.1-2),
 * batched over T transport blocks with one scrambling init each.  Packed bit words: bit k of
 * word w = element 32w + k. */

/* gen_nrPRBS (py5gphy/common/nrPRBS.py:5-25) of every TB: words [T][ldw] uint32 receive
 * c(0 .. nbits-1) for c_init = cinit[t] (cinit: DEVICE array of T values). */
int ldpc5g_prbs(const uint32_t* cinit, int32_t T, int64_t nbits, uint32_t* words, int64_t ldw,
                void* stream);

/* Modulation ids: the order Qm for QPSK..1024QAM, 1 for BPSK and LDPC5G_PI2_BPSK for pi/2-BPSK
 * (nrModulation.py:14-42 / nr_Demodulation.py:30-43 accept all seven). */
#define LDPC5G_PI2_BPSK (-1)

/* Scrambling + modulation mapper (nr_pdsch_process.py:17-25, nrModulation.py:4-42), mod = 1, -1,
 * 2, 4, 6, 8, 10: bits [T][ldb] int8 (nbits each, a multiple of Qm) XOR prbs words (NULL: no
 * scrambling) -> complex64 symbols [T][ldsym] (float2), bit-exact with the reference's float32
 * arithmetic (pi/2-BPSK: odd symbol index within each row rotated, :17-21). */
int ldpc5g_scramble_modulate(const int8_t* bits, int64_t ldb, const uint32_t* prbs, int64_t ldw,
                             int32_t T, int64_t nbits, int32_t mod, void* sym, int64_t ldsym,
                             void* stream);

/* Soft demodulation (nr_Demodulation.py:12-46, demod_{bpsk,pi2_bpsk,qpsk,16qam,64qam,256qam,
 * 1024qam}.py) + LLR descrambling (nr_pdsch.py:268-274): symbols [T][ldsym] complex64
 * (sym_dtype LDPC5G_F32) or complex128 (LDPC5G_F64), noise variances [T][ldnv] float32 -> LLRs
 * [T][ldllr] (nsym*Qm each), multiplied by 1 - 2c(n) when prbs is not NULL.  The arithmetic
 * follows the reference's operation order in the symbols' precision: float64 for complex128;
 * float32 for complex64 with every constant (k*A, c*A, threshold*A) rounded to float32 first, as
 * numpy >= 2 evaluates demod_*.py then.  llr_dtype LDPC5G_F32 always works; LDPC5G_F64 is accepted
 * for BPSK on complex128 input, whose reference LLRs are float64 (demod_bpsk.py:9). */
int ldpc5g_demod_descramble(const void* sym, int32_t sym_dtype, int64_t ldsym,
                            const float* noise_var, int64_t ldnv, const uint32_t* prbs,
                            int64_t ldw, int32_t T, int64_t nsym, int32_t mod, void* llr,
                            int32_t llr_dtype, int64_t ldllr, void* stream);

/* ================================================ gather records (multi-GPU)
 * Record r (a row of rec, stride ldr bytes) = the nbits int8 bits of row r of `bits` (values 0/1)
 * packed in np.packbits order (bit i -> byte i/8, bit 7 - i%8, tail zero-padded), then
 * status[r] (one byte, if status != NULL), then iters[r] (int32 little-endian, if iters != NULL).
 * One record per codeblock (bits = its K info bits) or per transport block (its tbblk + CRC
 * flag): a rank's results become one contiguous block for a single gather.  unpack reverses it;
 * any of bits / status / iters may be NULL there to skip that field.  No reference counterpart
 * (the reference runs in one process); the unpacked bits are the reference's blkandcrc / tbblk
 * (nr_ldpc_decode.py:47-49, nr_dlsch_decode.py:103-109). */
int ldpc5g_pack_records(const int8_t* bits, int64_t ldb, int32_t R, int64_t nbits,
                        const uint8_t* status, const int32_t* iters, uint8_t* rec, int64_t ldr,
                        void* stream);
int ldpc5g_unpack_records(const uint8_t* rec, int64_t ldr, int32_t R, int64_t nbits, int8_t* bits,
                          int64_t ldb, uint8_t* status, int32_t* iters, int64_t fstride,
                          void* stream);   /* status / iters of record r at [r * fstride] */

/* Message of the last failed call on this thread ("" if none). */
const char* ldpc5g_last_error(void);

/* Library version string. */
const char* ldpc5g_version(void);

/* Diagnostics: decoder workgroups that can be resident on one CU (HIP occupancy calculator) for
 * (bgn, llr_dtype, schedule).  No reference counterpart. */
int ldpc5g_dec_blocks_per_cu(int32_t bgn, int32_t llr_dtype, int32_t schedule);

/* ---- the multi-workgroup float64 decoder (few large codeblocks per call).
 * ldpc5g_decode_ms / ldpc5g_decode_ms_host / ldpc5g_sch_decode with float64 flooding and at most
 * ~24 codeblocks of Zc >= 64 (the per-codeblock drop-ins' shape) run each codeblock over W (9-18)
 * workgroups, one per CU, that synchronise through global memory twice per iteration.  It assumes:
 *   - co-residency: a codeblock's W workgroups run at the same time.  Workgroups take their
 *     (codeblock, part) by arrival ticket, so one launch never waits on itself, and launches use at
 *     most 7/8 of the device's CUs; but a kernel of another library or process that holds CUs
 *     indefinitely (a persistent kernel) could keep parts from starting.  A barrier wait therefore
 *     gives up after 4 s: the codeblock is returned with status 0 and iters -1 (never silently
 *     wrong), the device's timeout count grows (below), and the library stays usable;
 *   - serialisation: split launches of one device are chained by one hidden event (they share a
 *     per-device sync area and scratch), so they run one after another whatever their streams;
 *   - the first split launch on a device, and one needing more scratch, allocate (hipMalloc /
 *     hipMemset / a device synchronisation, or an event wait + hipFree when growing): not capturable.
 *     A stream in capture (hipStreamIsCapturing) never takes this path — such launches run the
 *     one-workgroup-per-codeblock kernels instead (same results, bit for bit).
 * ldpc5g_split_timeouts: the number of codeblocks of the current device whose split decode timed
 * out since the process started (waits for the device's last split launch).  No reference
 * counterpart. */
int ldpc5g_split_timeouts(uint32_t* count);

#ifdef __cplusplus
}
#endif

#endif /* LDPC5G_H */
