// cal_internal.hpp -- shared types of the MI355X CA-Lanczos library.
//
// Data layout in HBM:
//  * A: local CSR (int32 rowptr/col, fp64 val) + "row blocks" for the
//    LDS-staged CSR-stream SpMV (<= 256 rows and <= 2048 nonzeros each).
//  * every n-vector (columns of V, Q, scratch) lives in a column-major buffer
//    with leading dimension ld = roundup(n_local + nghost, 64): the ghost
//    entries of a slab live right after its local entries, so a halo
//    exchange writes straight into the column the SpMV gathers from.
#pragma once

#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <cstdint>
#include <cstdlib>
#include <functional>
#include <string>
#include <vector>

#include "../../include/calanczos.h"

// rocprofv3 --marker-trace range (host time) for the scope of one object
struct RoctxRange {
    explicit RoctxRange(const char* msg) { roctxRangePushA(msg); }
    ~RoctxRange() { roctxRangePop(); }
    RoctxRange(const RoctxRange&) = delete;
    RoctxRange& operator=(const RoctxRange&) = delete;
};

namespace cal {

constexpr int kMaxSeg = 4;

// A concatenation of up to kMaxSeg column-major segments ("[Q_p | X]").
struct Panel {
    const double* ptr[kMaxSeg];
    int64_t ld[kMaxSeg];
    int ncol[kMaxSeg];
    int nseg;
    int total;
};

struct PanelOut {
    double* ptr[kMaxSeg];
    int64_t ld[kMaxSeg];
    int ncol[kMaxSeg];
    int nseg;
    int total;
};

inline Panel panel() {
    Panel p{};
    return p;
}
inline Panel& panel_add(Panel& p, const double* ptr, int64_t ld, int ncol) {
    if (ncol <= 0) return p;
    p.ptr[p.nseg] = ptr;
    p.ld[p.nseg] = ld;
    p.ncol[p.nseg] = ncol;
    p.nseg++;
    p.total += ncol;
    return p;
}
inline PanelOut panel_out(double* ptr, int64_t ld, int ncol) {
    PanelOut p{};
    p.ptr[0] = ptr;
    p.ld[0] = ld;
    p.ncol[0] = ncol;
    p.nseg = 1;
    p.total = ncol;
    return p;
}

// SpMV launch description (local CSR; x/y are columns with ghost space).
struct SpmvArgs {
    const int* rowptr;
    const int* col;
    const double* val;
    const int* blk;
    int nblk;
    const double* x;
    double* y;
    const double* xprev;  // modified Newton basis, complex shift
    double shift;         // y = A x - shift * x
    double im2;           //     + im2 * xprev
    int mode;             // 0: y = A x, 1: shifted, 2: shifted + im2 term,
                          // 3: y = A (x / sqrt(*xnrm)) (normest; each gathered x_j divided)
    const double* xnrm = nullptr;
    int xcd;              // XCD-contiguous block order (set by launch_spmv)
    int nt = 0;           // col / val loaded non-temporally (matrix larger than the Infinity Cache)
};

// Row-pattern storage ("PSR"): row r is pattern pat[r], a sequence of
// (col - row, value) pairs in increasing column order held in a small table.
// Lossless and summed in CSR order, so SpMV results are bit-identical to CSR.
struct PatArgs {
    const uint16_t* pat;
    const int2* pinfo;     // (start, len) per pattern; empty rows -> sentinel
    const int* pdelta;
    const double* pval;
    int64_t n;
    int nblk;              // ceil(n / 256)
    const double* x;       // local origin (offsets may reach into the halo)
    double* y;
    const double* xprev;
    double shift, im2;
    int mode;              // as SpmvArgs
    int maxlen;            // 1..8 exact, else 16 / 32
    int npat, nent;        // table sizes (LDS-resident when small)
    // pair patterns (k_spmv_pair): rows 2t, 2t+1 share one merged pattern
    const uint16_t* ppat;  // per pair; kPairSplit -> per-row fallback
    const int2* ppinfo;    // (start, len) per pair pattern
    const int* ppoff;      // (offset << 2) | used-by-row-2t | used-by-row-2t+1 << 1
    const double2* ppval;  // (value for row 2t, value for row 2t+1)
    int nppat, npent, pmaxlen;
    int pcanon;            // every pair pattern has exactly pmaxlen entries (canonical slots)
    int pslot[8];          // canonical slot offsets (the matrix's distinct col - row, ascending)
    int pmid = -1;         // pmaxlen / 2 when slots pmid - 1, pmid, pmid + 1 are the offsets -1, 0, +1
    int64_t xlo, xhi;      // addressable range of a vector column around its origin
    // plane march (k_resid_planes): the canonical slots' values per row
    // pattern with +0.0 where the row has no entry (npat x pmaxlen), the
    // plane stride P = pslot[pmaxlen-1] = -pslot[0] and the in-plane reach H
    // (the other slots' largest |offset|, rounded up to even); plane_P = 0:
    // the matrix has no plane structure for it
    const double* rzval = nullptr;
    const uint8_t* rzmask = nullptr;  // bit e: the row pattern has an entry at slot e
    // the row pattern ids as bytes (npat <= 256; the plane march's keys)
    const uint8_t* rowkey8 = nullptr;
    // uniform slot values (every row with an entry at slot e has the value
    // cval[e], as in the Laplacians): the plane march keys each row by its
    // slot mask byte (rowmask) and takes the values from cval
    const uint8_t* rowmask = nullptr;
    const uint32_t* wavemask = nullptr;  // DevMatrix::wavemask
    int cuniform = 0;
    double cval[8] = {};
    int64_t plane_P = 0;
    int plane_H = 0;
    int64_t ld = 0;  // the vector columns' leading dimension (the descriptor's range)
    // two-range launch (pair kernel): compact pair index t >= gap_at maps to
    // stored pair t + gap, i.e. rows [0, 2 gap_at) and [2 (gap_at + gap),
    // 2 gap + n) relative to the origin; n counts the rows of both ranges
    int64_t gap_at = 0, gap = 0;
};
constexpr int kPairSplit = 0xFFFF;
// the plane march: rows of a plane per block (4 waves x 64 lanes x 2 rows)
constexpr int kPlaneBlockRows = 512;

struct DevMatrix {
    int64_t n_local = 0, n_global = 0, row0 = 0, nnz = 0, nghost = 0;
    // Stored rows: n_rows = ext_off + n_local + right ghost rows.  With the
    // CA matrix-powers kernel (mpk) a slab also stores the rows of its
    // (depth-1)-deep ghost zone, fetched from the owners at setup, so the s
    // powers of one outer iteration need one deep halo exchange instead of s
    // (DESIGN.md §4).  ext_off (even, for the pair kernel) counts the stored
    // rows before the first local row, including one empty dummy row when
    // the ghost count is odd; columns stay relative to the local origin.
    int64_t n_rows = 0, ext_off = 0, nnz_loc = 0;
    bool mpk = false;
    int mpk_depth = 1;                   // stored ghost depth D (powers per exchange)
    int64_t band_l = 0, band_r = 0;      // global max (row - min col), (max col - row)
    int64_t ext_lo = 0, ext_hi = 0;      // global rows of the first / one past the last real stored row
    int ext_dummy = 0;                   // stored row 0 is an empty dummy row
    std::vector<int64_t> slabs;          // slab starts of every rank (+ n_global)
    int* rowptr = nullptr;
    int* col = nullptr;    // local column ids relative to the local origin
    double* val = nullptr;
    int* blk = nullptr;
    int nblk = 0;
    int nit = 1;     // ceil(max row-block nonzeros / 256): SpMV unroll depth
    int64_t ld = 0;  // leading dimension of every n-vector buffer
    int64_t lpad = 0;  // offset of the local origin inside each vector column
    // row-pattern format (chosen automatically when the table is small)
    bool use_pat = false;
    uint16_t* pat = nullptr;
    int2* pinfo = nullptr;
    int* pdelta = nullptr;
    double* pval = nullptr;
    int npat = 0, nent = 0, maxlen = 0;
    // pair patterns (two rows per lane, 16-B x loads; built with the row patterns)
    bool use_pair = false;
    uint16_t* ppat = nullptr;
    int2* ppinfo = nullptr;
    int* ppoff = nullptr;
    double2* ppval = nullptr;
    int nppat = 0, npent = 0, pmaxlen = 0;
    int64_t npsplit = 0;
    bool pcanon = false;
    int pslot[8] = {};
    // plane-march residual table (PatArgs::rzval; single rank, no halos)
    double* rzval = nullptr;
    uint8_t* rzmask = nullptr;
    uint8_t* rowkey8 = nullptr;
    uint8_t* rowmask = nullptr;
    // per plane z (0 .. nz, the last one zero) and 512-row block xy of the
    // plane march: byte w = OR over the 128 rows of wave w of the slots those
    // rows lack (rows past n lack every slot); the march masks only those
    // slots (kernels.hip, PlaneMarch)
    uint32_t* wavemask = nullptr;
    bool cuniform = false;
    double cval[8] = {};
    int64_t plane_P = 0;
    int plane_H = 0;
    // halo plan (distributed); ghost entries grouped by owning peer
    std::vector<int> peers;              // neighbour ranks
    std::vector<int64_t> recv_off;       // ghost destination per peer, relative to the local origin
    std::vector<int64_t> recv_cnt;
    std::vector<int64_t> send_off;       // offset into send index list
    std::vector<int64_t> send_cnt;
    int* send_idx = nullptr;             // device, local indices to pack
    int64_t send_total = 0;
    double* send_buf = nullptr;          // device pack buffer
};

struct Comm;  // comm.cpp
struct LanczosState;  // lanczos.cpp

// Launchers (kernels.hip).  All enqueue on `st` and return hipError_t.
hipError_t launch_spmv(const SpmvArgs& a, hipStream_t st);
hipError_t launch_spmv_pat(const PatArgs& a, hipStream_t st);
// C (wa x wb, column-major ldc = 16*ceil(wa/16)) partials; see kernels.hip.
struct GramPlan {
    int nta;    // A tiles of 16 columns
    int blocks;
    int64_t entries;  // per-block partial entries
};
GramPlan gram_plan(int wa, int wb, int64_t n);
hipError_t launch_gram(const Panel& A, const Panel& B, int64_t n, const GramPlan& pl, double* partial,
                       hipStream_t st);
// A'B and B'B in one pass (the row-staged Gram with B'B as an extra tile):
// pl.entries + 256 partial entries per block, B'B (ld 16) after A'B's
bool gram_bb_ok(int wa, int wb);
hipError_t launch_gram_bb(const Panel& A, const Panel& B, int64_t n, const GramPlan& pl, double* partial,
                          hipStream_t st);
struct ApplyPlan {
    int nty;
    int run;
    int blocks;
    bool gram;
    bool gramp;
    size_t lds_bytes;
    int64_t entries;  // per-block partial entries (gram + gramp)
};
ApplyPlan apply_plan(int wp, int wy, int64_t n, bool gram, int wq);
int apply_rows_max_wy(int wp);  // widest output chunk of the row-parallel store-only apply
bool apply_rows_ok(int wp, int wy);
// Y = P M (stored) and the Gram Qn'Y (partials of apply_gram_blocks(n) blocks
// x 256 entries, ldc 16) in one pass: wp <= 32, wy <= 16, Qn <= 16 columns
bool apply_gram_ok(int wp, int wy, int wq);
int apply_gram_blocks(int64_t n);
hipError_t launch_apply_gram(const Panel& P, const double* dM, int wp, int wy, const PanelOut& Y, const Panel& Qn,
                             int64_t n, double* partial, hipStream_t st);
// Y = P M (stored) and Y'Y as the 272-entry tile partials of the rowgram
// (P1 of orth_device) over *blocks blocks: wp <= 32, wy <= 16
bool apply_selfgram_ok(int wp, int wy);
hipError_t launch_apply_selfgram(const Panel& P, const double* dM, int wp, int wy, const PanelOut& Y, int64_t n,
                                 double* partial, int* blocks, hipStream_t st);
hipError_t launch_apply(const Panel& P, const double* dM, int wp, int wy, const PanelOut& Y, bool store,
                        int wq, int64_t n, const ApplyPlan& pl, double* partial, hipStream_t st);
hipError_t launch_reduce(const double* partial, int nparts, int64_t nent, double* out, hipStream_t st);
// one-pass block-upper Gram of w <= 128 columns of one buffer (k_gram_wide):
// gram_wide_entries(w) entries of gram_wide_blocks(n) block partials each
// (entry-major); entry e is G(i, j) with (i, j) from gram_wide_entry
hipError_t launch_gram_wide(const double* Q, int64_t ld, int w, int64_t n, double* partial, hipStream_t st);
int gram_wide_entries(int w);
int gram_wide_blocks(int64_t n);
void gram_wide_entry(int w, int e, int* i, int* j);
// hot-shape kernels (s <= 8): tile Gram (<= 16 columns + 1 extra) and the
// row-parallel apply with the fused LDS-transposed tile Gram.  Partials:
// 272 entries (16x16 tile Gram, then 16 extra-column products).
hipError_t launch_tilegram(const Panel& T, const double* E, int64_t n, int blocks, double* partial, hipStream_t st);
int rowapply_wpmax(int wp);
int rowapply_mout(int m);
// column pointers resolved on the host (kernel-argument arrays -> SGPR bases)
struct ColList {
    const double* p[17];
};
struct OutList {
    double* p[16];
};
// kind: 0 store, 1 store + Gram, 2 Gram only (pass A), 3 chained store (pass B).
// gate (kind 3): device flags; a nonzero gate[0] or gate[1] skips the store.
hipError_t launch_rowapply(const ColList& P, const double* dM, int wp, int m, const OutList& Y, int kind, int wq,
                           int64_t n, int blocks, double* partial, hipStream_t st, const double* gate = nullptr);
// s x s coefficients of the two-sweep block orthogonalisation (phase 0 after
// the P1 Gram, phase 1 after pass A); see kernels.hip k_orth_coef.
// Phase 1 with hout != nullptr also publishes out (R, RY, flags; 516
// doubles) to the host-mapped hout and then stores seq to *hseq (system-scope
// release): the host polls that word instead of copying and waiting.
hipError_t launch_orth_coef(int phase, const double* tile, double* st, double* mbuf, double* out, int w, int m,
                            int WP, int MO, int doreorth, double* hout, unsigned long long* hseq,
                            unsigned long long seq, hipStream_t stream);
// Grid of the row-parallel Gram sweeps (k_rowapply with GRAM): 4 blocks of
// 38 KB LDS per CU on 256 CUs.
#ifndef CAL_ROWGRAM_BLOCKS
#define CAL_ROWGRAM_BLOCKS 1024
#endif
constexpr int kRowGramBlocks = CAL_ROWGRAM_BLOCKS;
hipError_t launch_rowgram(const ColList& P, int nt, bool has_extra, int64_t n, int blocks, double* partial,
                          hipStream_t st);
// pass B (w = 9, m = 8) fused with G = [Qp | Q_new | Qold]' Q_new (kernels.hip
// k_passb_wide): passb_wide_tiles(wold) 16-column groups, at most
// kPassbWideMaxTiles; partial entries j (16 tiles) + a, j < 8
constexpr int kPassbWideMaxTiles = 12;
int passb_wide_tiles(int wold);
hipError_t launch_passb_wide(const ColList& P, const double* dM, const OutList& Y, const Panel& Qold, int64_t n,
                             int blocks, double* partial, const double* gate, hipStream_t st);
hipError_t launch_dot(const double* x, const double* y, int64_t n, double* partial, int blocks,
                      hipStream_t st);
int dot_blocks(int64_t n);
hipError_t launch_axpy_sub(double* y, const double* x, double a, int64_t n, hipStream_t st);  // y -= a*x
hipError_t launch_div(double* y, const double* x, double b, int64_t n, hipStream_t st);      // y = x / b
hipError_t launch_form_projM(const double* G, int ldg, int w, int m, double* M, hipStream_t st);
// y -= a * x, a = *pa (take_sqrt: sqrt(*pa)) read on the device
// one step of the Newton prologue's recurrence, single rank (kernels.hip
// k_pro_*): r -= sqrt(*pb_prev) qprev (qprev may be null), alpha = r'q ->
// *d_alpha, r -= alpha q, beta^2 = r'r -> *d_beta2, qnext = r / beta; part:
// 2 dot_blocks(n) doubles
// normest's iteration tail, single rank: dst[0] = x'x, dst[1] = y'y, x /= sqrt(x'x)
// (part: 2 dot_blocks(n) doubles)
hipError_t launch_normest_norms(double* x, const double* y, int64_t n, double* part, double* dst, hipStream_t st);
// the same norms without rescaling x (the next S*x divides in its gathers: MODE 3)
hipError_t launch_normest_norms_only(const double* x, const double* y, int64_t n, double* part, double* dst,
                                     hipStream_t st);
hipError_t launch_pro_step(double* r, const double* qprev, const double* pb_prev, const double* q, double* qnext,
                           int64_t n, double* part, double* d_alpha, double* d_beta2, hipStream_t st);
hipError_t launch_axpy_sub_dev(double* y, const double* x, const double* pa, bool take_sqrt, int64_t n,
                               hipStream_t st);
hipError_t launch_div_sqrt(double* y, const double* x, const double* nn, int64_t n, hipStream_t st);  // y = x / sqrt(*nn)
hipError_t launch_abs_rowsum(const int* rowptr, const double* val, int64_t n, double* y, hipStream_t st);
hipError_t launch_gather(double* dst, const double* src, const int* idx, int64_t cnt, hipStream_t st);
// fused SpMV + Ritz residual partials for one Ritz pair (diagnostics)
// Gram A'B (A <= 128 columns, B <= 16) reduced, all-reduced and copied to
// h_dst (ld *ldc) asynchronously: valid after the stream's next wait
// (part: the block partials' scratch, gram_plan blocks x entries doubles; default c->d_partial)
// bb: B'B too (gram_bb_ok), 256 entries (ld 16) at d_dst / h_dst + 16 *ldc * 16 (after A'B)
int gram_async(cal_ctx* c, int64_t n, const Panel& A, const Panel& B, double* d_dst, double* h_dst, int* ldc,
               double* part = nullptr, bool bb = false);
int spmv_pair_resid_blocks(const PatArgs& a);
hipError_t launch_spmv_pair_resid(const PatArgs& a, double lr, double* partial, hipStream_t st);
// the same for npr real Ritz pairs in one launch: x_i = X + col[i] * ldx,
// l_i = lam[i]; sums of pair i at partial[(2 out[i] + e) * pstride + block]
hipError_t launch_spmv_pair_resid_multi(const PatArgs& a, const double* X, int64_t ldx, const int* col,
                                        const double* lam, const int* out, int npr, double* partial,
                                        int64_t pstride, hipStream_t st);
int spmv_resid_pair_multi_dev(cal_ctx* c, const double* X, int64_t ldx, const int* col, const double* lam,
                              const int* out, int npr, double* partial, int64_t pstride);
int spmv_pair_resid_multi_blocks(const PatArgs& a);
int spmv_resid_pair_multi_blocks(cal_ctx* c);  // its grid (0: no pair path)
// store-only Y = P M on the matrix cores (one segment each, 16-B aligned,
// Y not aliasing P; M wp x wy column-major on the device)
bool apply_mt_ok(int wp, int wy);
hipError_t launch_apply_mt(const double* P, int64_t ldp, const double* dM, int wp, int wy, double* Y, int64_t ldy,
                           int64_t n, hipStream_t st);
// Ritz residual partials of a real Ritz value on the pair patterns (local
// rows; x's halo already exchanged): *blocks = 0 when the path does not apply
int spmv_resid_pair_dev(cal_ctx* c, const double* x, double lr, double* partial, int* blocks);
int spmv_resid_pair_blocks(cal_ctx* c);
hipError_t launch_spmv_resid(const SpmvArgs& a, const double* xi, double lr, double li, int64_t nrows,
                             double* partial, int blocks, hipStream_t st);

// ---- Householder TSQR (tsqr.hip / tsqr.cpp) ------------------------------
constexpr int kTsqrMaxCols = 33;
struct TsqrCols {
    const double* p[kTsqrMaxCols];
};
struct TsqrQ {
    double* p[32];
};
// One level of the TSQR tree.  Level 0 reads the panel (direct columns, or
// Z = P M formed per row with M wp x m column-major); higher levels read the
// stack of the level below: one m x m column-major block per tile (block
// layout).  UP writes each tile's R as a block of `out`; DOWN reads the
// tile's S block from `S` (null at the root: the sign fix) and writes Q rows
// (level 0: TsqrQ columns; higher levels: `out` in block layout).
struct TsqrLevelArgs {
    int64_t rows = 0;
    int m = 0;
    int wp = 0;
    const double* M = nullptr;
    const double* in = nullptr;
    double* out = nullptr;
    const double* S = nullptr;
    const double* M2 = nullptr;  // formed mode: Z = (P M) + P(:, 0:w2) M2 (w2 x m)
    int w2 = 0;
    // level 0: UP stores each tile's factored registers (reflectors and R,
    // 64 * RPL * MM doubles per tile, lane-contiguous) and tau / beta (MM
    // each); DOWN (src 3) reloads them instead of re-forming and re-factoring
    double* V = nullptr;
    double* tb = nullptr;
};
int tsqr_mm(int m);          // register tile width (8, 16, 32; 0: m > 32)
int tsqr_tile_rows(int m);   // rows per tile (4096 / tsqr_mm)
bool tsqr_form_ok(int wp, int m);
// src: 0 stack, 1 direct columns, 2 formed, 3 (DOWN at level 0) the reflectors UP stored
hipError_t launch_tsqr(bool down, int src, const TsqrLevelArgs& a, const TsqrCols& P, const TsqrQ& Q,
                       hipStream_t st);


// ---- projectAndNormalize with the fused TSQR (tsqr_fold.hip) ----------------
// Workspace of one fused block (8-wide register tiles): level 0 (n0 tiles of
// 256 rows: factored tiles V0 / tau-beta tb0, R factors R0), the upper
// levels L = 1 .. nlev (nu[L-1] tiles of 64 R factors of the level below:
// reflectors Vu, R factors Ru, WY matrices Mu; level nlev is the root, one
// tile; Rroot_m its R with ld m), the P1 tile C, K (9 x 8), the flags
// (out[512..515]), the C2 = Qp'Y partials (72 x nblk, entry-major; red_out:
// where level 1 reduces them, or null) and the root's S (Stop, ld lds).
// largest accepted loss-of-orthogonality estimate of the fused TSQR (its
// default; cal_set_tsqr_fold_tol)
constexpr double kFoldTol = 1e-14;
struct FoldArgs {
    int64_t n = 0;
    double tol = kFoldTol;
    int m = 0, w = 0, nblk = 0, n0 = 0, nlev = 0;
    int nu[3] = {0, 0, 0};
    const double* C = nullptr;  // the reduced P1 tile (272 doubles): C = Qp'X is read from it
    const double* flags = nullptr;
    const double* K = nullptr;
    double *V0 = nullptr, *tb0 = nullptr, *R0 = nullptr;
    double* Vu[3] = {nullptr, nullptr, nullptr};
    double* Ru[3] = {nullptr, nullptr, nullptr};
    double* Mu[3] = {nullptr, nullptr, nullptr};
    double* Rroot_m = nullptr;
    double* partial = nullptr;
    double* red_out = nullptr;
    const double* Stop = nullptr;
    int lds = 8;
};
int fold_tiles(int64_t n);                 // level-0 tiles
int fold_blocks(int64_t n);                // k_fold_up / k_fold_down blocks
std::vector<int> fold_levels(int64_t n);   // tiles of the upper levels (the last: the root)
bool fold_shape_ok(int64_t n, int m, int w);
size_t fold_l0_tile_doubles();  // one level-0 tile
size_t fold_tile_doubles();     // one upper-level tile (512 x 8)
hipError_t launch_fold_up(const ColList& P, const FoldArgs& a, hipStream_t st);
// levels 1 .. upto (-1: up to the root)
hipError_t launch_fold_tree(const FoldArgs& a, hipStream_t st, int upto = -1);
hipError_t launch_fold_reduce(const double* partial, int nparts, double* out, hipStream_t st);  // the 72 C2 entries
// k_fold_coef1: T1 the reduced P1 tile, G the up launch's Gram tile, Rtop the
// root R (ld ldr); writes out (R, RY, flags), S_top (Sbuf ld 8, Sm ld m), K
// and publishes R / RY / flags to hout, then seq to *hseq
hipError_t launch_fold_coef1(const double* T1, const double* G, const double* Rtop, int ldr, double* out,
                             double* Sbuf, double* Sm, double* Kbuf, int w, int m, int doreorth, double nglob,
                             double tol, double* hout, unsigned long long* hseq, unsigned long long seq,
                             hipStream_t st);
// one rank: the root level and k_fold_coef1's algebra in one block (the
// root's R is its own, ld 8)
hipError_t launch_fold_root(const FoldArgs& a, const double* T1, const double* G, double* out, double* Sbuf,
                            double* Sm, double* Kbuf, int w, int doreorth, double nglob, double* hout,
                            unsigned long long* hseq, unsigned long long seq, hipStream_t st);
hipError_t launch_fold_down(const ColList& P, const OutList& Q, const FoldArgs& a, hipStream_t st);


}  // namespace cal

// Per-launch kernel timer (HIP events on the launching stream).
struct CalTimerRec {
    int kind;  // 0 spmv, 1 gram, 2 apply, 3 other, 4 allreduce (RCCL), 5 halo exchange (RCCL)
    hipEvent_t a, b;
    double bytes;  // the launch's algorithmic HBM bytes, 0 if not stated
};

struct cal_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    hipStream_t aux_stream = nullptr;  // second stream of the diagnostics (lanczos.cpp diag_launch), lazy
    std::string err;
    cal::DevMatrix A;
    bool has_A = false;
    uint64_t A_gen = 0;  // matrix uploads so far (keys what was captured against A)
    int64_t stat_spmv_rows = 0;  // rows computed by SpMV launches (cal_comm_stats)

    // reduction scratch
    double* d_partial = nullptr;
    size_t partial_cap = 0;  // doubles
    double* d_red = nullptr;
    double* h_red = nullptr;  // pinned
    size_t red_cap = 0;       // doubles
    double* d_small = nullptr;  // small matrices (M operands)
    double* h_small = nullptr;  // pinned staging for d_small
    size_t small_cap = 0;
    bool small_pending = false;  // an async copy out of h_small may be in flight
    double* d_scratch = nullptr;  // host-pointer entry points (tier-1 calls)
    size_t scratch_cap = 0;

    // generic device workspace (n-vector columns)
    double* d_work = nullptr;
    int work_cols = 0;
    int64_t work_ld = 0;

    cal::LanczosState* lz = nullptr;
    cal::Comm* comm = nullptr;

    bool timing = false;
    std::vector<CalTimerRec> timers;
    std::vector<hipEvent_t> event_pool;

    int spmv_format = 0;  // 0 auto, 1 CSR, 2 row-pattern (applies at the next set_matrix)
    int mpk_depth_req = 8;
    // schedule of the last powers_dev call (cal_mpk_schedule): 0 one halo
    // exchange per SpMV, 1 one deep exchange, 2 deep exchange on the RCCL
    // stream overlapped with the interior powers, 3 split schedule with a
    // synchronous exchange, 4 the host-staged twin of 2; -1 none yet
    int powers_launches = 0;   // SpMV-class launches of the last powers_dev call
    int powers_schedule = -1;  // ghost depth of the distributed matrix-powers kernel (next set_matrix; 1 = off)
    bool orth_coef_device = true;  // block-orth s x s algebra on the device (blockorth.cpp)
    // set by lanczos_step: work to enqueue after a block orthogonalisation is
    // enqueued and before the host waits for its R (orth_device)
    std::function<int()> pre_wait;
    // 'full' orthogonalisation (lanczos_step): the local block's pass B also
    // forms the next projection's Gram [Qp | Q_new | Qold]' Q_new
    // (k_passb_wide); want/qold set by the caller, ready once the reduced
    // Gram's copy to h_pbw is enqueued (pbw_event after it)
    struct {
        bool want = false, ready = false;
        cal::Panel qold{};
        int ntw = 0;
        double* d = nullptr;
        double* h = nullptr;
        size_t cap = 0;
        hipEvent_t ev = nullptr;
    } pbw;
    bool orth_redone = false;  // the last block was redone on the host path
    hipEvent_t orth_event = nullptr;
    // device-coefficient block orthogonalisation: the pinned host-mapped
    // result page the phase-1 kernel publishes R / RY / flags into (h_pub,
    // device alias d_pub; the sequence word follows the 516 doubles)
    double* h_pub = nullptr;
    double* d_pub = nullptr;
    unsigned long long pub_seq = 0;
    // normalize (tsqr.m) backend: 0 "auto" (Householder TSQR for the tier-1
    // calls, CholQR2 in the CA-Lanczos loop with TSQR when its Cholesky
    // fails), 1 "tsqr" (Householder TSQR everywhere), 2 "cholqr2" (CholQR2
    // everywhere, shifted CholQR3 when its Cholesky fails)
    int normalize_kind = 0;
    bool tier1 = false;  // inside a host-pointer (tier-1) entry point (api.cpp)
    double* d_tsqr = nullptr;  // TSQR tree workspace
    size_t tsqr_cap = 0;
    double* d_tsqrv = nullptr;  // level-0 reflectors of the TSQR (tsqr_tree.cpp)
    size_t tsqrv_cap = 0;
    double* d_zbuf = nullptr;  // n x m block of the TSQR paths (blockorth.cpp)
    size_t zbuf_cap = 0;
    double* d_fold = nullptr;  // fused TSQR workspace (blockorth.cpp pn_tsqr_fold)
    size_t fold_cap = 0;
    long fold_runs = 0, fold_declined = 0;  // fused-TSQR blocks run / declined (explicit-Z path taken)
    double fold_last_est = 0.0;             // the last block's loss-of-orthogonality estimate
    double fold_tol = cal::kFoldTol;        // its acceptance threshold (cal_set_tsqr_fold_tol)
    // the asynchronous normest (lanczos.cpp normest_async_*): its stream,
    // completion event, device scratch (x, Sx, partials, norms) and pinned
    // norms, grown to the matrix once and reused by every solve
    hipStream_t nest_stream = nullptr;
    hipEvent_t nest_event = nullptr;
    double* d_nest = nullptr;
    double* h_nest = nullptr;
    size_t nest_cap = 0;
    // its chunks as replayed HIP graphs (one host launch per chunk, not ~50):
    // [0] the first chunk, [1] the later ones; each valid for the key it was
    // captured with (scratch, matrix arrays, sizes)
    hipGraphExec_t nest_exec[2] = {nullptr, nullptr};
    std::vector<int64_t> nest_key[2];
    // the test build only (CAL_TEST_HOOKS): R of ca_lanczos's first block
    // (normalize, ca_lanczos.m:176), read back by cal_test_first_block_R
    std::vector<double> test_R1;
};

// ---- helpers shared by the host-side translation units -----------------
namespace cal {

int set_error(cal_ctx* c, int code, const std::string& msg);
int hip_fail(cal_ctx* c, hipError_t e, const char* what);

#define CAL_HIP(ctx, expr)                                  \
    do {                                                    \
        hipError_t _e = (expr);                             \
        if (_e != hipSuccess) return cal::hip_fail((ctx), _e, #expr); \
    } while (0)
// a small launch (reduction, coefficient step, vector op, result copy)
// bracketed by the "other" kernel timer when timing is on
#define CAL_HIP_OTHER(ctx, expr)                                            \
    do {                                                                    \
        const int _t = cal::timer_begin((ctx), 3);                          \
        hipError_t _e = (expr);                                             \
        cal::timer_end((ctx), _t);                                          \
        if (_e != hipSuccess) return cal::hip_fail((ctx), _e, #expr);       \
    } while (0)
#define CAL_TRY(expr)             \
    do {                          \
        int _s = (expr);          \
        if (_s < 0) return _s;    \
    } while (0)

// rowptr/col/val: n_rows stored rows, the local ones starting at stored row
// ext_off; col: ids relative to the local origin (negative = left halo);
// lpad/rext: halo extent on each side of the local rows in a vector column.
// Pinned host-mapped result page of the device block orthogonalisation:
// 516 doubles (R, RY, flags) then the 8-byte sequence word.
constexpr int kPubDoubles = 520;
int ensure_pub(cal_ctx* c);

int upload_matrix(cal_ctx* c, int64_t n_rows, int64_t ext_off, int64_t n_local, int64_t n_global, int64_t row0,
                  int64_t nghost, int64_t lpad, int64_t rext, const std::vector<int>& rowptr,
                  const std::vector<int>& col, const double* val);
// Row-pattern SpMV over stored rows [o, o+len) (o even); x, y at the local origin.
int spmv_range(cal_ctx* c, int64_t o, int64_t len, const double* x, double* y, int mode, double shift, double im2,
               const double* xprev);
// The s matrix powers Y[j] = (A - shift_j I) x_j (+ im2_j xprev_j), x_0 = q,
// x_j = Y[j-1] (matrix_powers_{monomial,newton}.m): with the CA
// matrix-powers kernel when the matrix has one (one deep halo exchange),
// otherwise one halo exchange per SpMV.  shift/im2/xprev may be null.
int powers_dev(cal_ctx* c, int s, const double* q, double* const* Y, const double* shift, const double* im2,
               const double* const* xprev);
// Halo exchange of the d-deep ghost zone of x (contiguous row ranges; mpk only).
int halo_exchange_deep(cal_ctx* c, double* x, int d, hipStream_t st);
// copy the n local rows of m columns (leading dimension ld) on the context
// stream; src/dst are local-origin pointers (a whole-column copy from there
// would run lpad entries past the last column)
inline hipError_t copy_cols(cal_ctx* c, double* dst, const double* src, int64_t ld, int64_t n, int m) {
    if (n <= 0 || m <= 0) return hipSuccess;
    return hipMemcpy2DAsync(dst, ld * sizeof(double), src, ld * sizeof(double), n * sizeof(double), m,
                            hipMemcpyDeviceToDevice, c->stream);
}
// pointer to column j of a vector buffer laid out with A.ld / A.lpad
inline double* vcol(const cal_ctx* c, double* base, int64_t j) { return base + j * c->A.ld + c->A.lpad; }
// A/B switches of the test build (libcalanczos_testhooks.so: lanczos.cpp,
// blockorth.cpp and runtime.cpp compiled -DCAL_TEST_HOOKS), read per call;
// the production library reads no such variable.
inline bool test_switch(const char* name) {
#ifdef CAL_TEST_HOOKS
    return std::getenv(name) != nullptr;
#else
    (void)name;
    return false;
#endif
}
// Device scratch allocation.  The test build fills every new buffer with NaN
// (all-ones bytes, then a device sync): a kernel that reads scratch it did
// not write first returns NaN there instead of a previous allocation's data.
hipError_t scratch_malloc(void** p, size_t bytes);
int ensure_partial(cal_ctx* c, size_t doubles);
int ensure_scratch(cal_ctx* c, size_t doubles);
int ensure_red(cal_ctx* c, size_t doubles);
int ensure_small(cal_ctx* c, size_t doubles);
int ensure_work(cal_ctx* c, int cols, int64_t ld);
double* work_col(cal_ctx* c, int j);

// timer bracket: returns an index, -1 if timing is off
int timer_begin(cal_ctx* c, int kind, double bytes = 0.0);
// the same on another stream (the halo exchange on the communicator's stream)
int timer_begin_on(cal_ctx* c, int kind, hipStream_t st);
void timer_end_on(cal_ctx* c, int idx, hipStream_t st);
void timer_end(cal_ctx* c, int idx);

// Device block operations (blockorth.cpp).  All matrices column-major; n is
// the number of (local) rows of the panels.
// Gram: out (wa x wb, ld wa) = A^T B (allreduced across ranks), on host.
int gram_host(cal_ctx* c, int64_t n, const Panel& A, const Panel& B, double* out);
// Apply: Y = P * M (M host, wp x wy col-major).  Optional gram (Y^T Y, wy x wy)
// and gramp (Psub^T Y, wq x wy where Psub = first wq columns of P), on host.
int apply_host(cal_ctx* c, int64_t n, const Panel& P, const double* M, int wy, const PanelOut* Y, double* gram,
               int wq, double* gramp);
// Y = P * M, M (wp x wy) already on the device; store only
int apply_dev(cal_ctx* c, int64_t n, const Panel& P, const double* dM, int wy, const PanelOut& Y);
// Reorthogonalisation helpers used by the driver and the C ABI.
struct PNResult {
    bool reorth = false;
    int rank = 0;
    bool chol_shifted = false;
};
// CholQR2 normalise of the n x m panel X into Qout, R (m x m) on host.
// p1_blocks: X'X's tile partials already in d_partial (blockorth.cpp orth_device)
int normalize_dev(cal_ctx* c, int64_t n, const Panel& X, const PanelOut& Qout, double* R, double tol, int* rank,
                  bool* shifted, int p1_blocks = 0);
// projectAndNormalize of X (n x m) against one block Qp (n x w): QZ into Qout,
// Rq (w x m) and R (m x m) on host.  Mirrors projectAndNormalize.m:3-90.
// G1_pre (optional, wide Qp only): [Qp | X]' X ((w+m) x m), already formed
// (the local block's k_passb_wide): the Gram sweep is skipped.
int project_and_normalize_dev(cal_ctx* c, int64_t n, const Panel& Qp, const Panel& X, bool doreorth,
                              const PanelOut& Qout, double* Rq, double* R, PNResult* res,
                              const double* G1_pre = nullptr);
// project.m:7-58 on device blocks (block MGS across blocks, CGS within); X in place.
int project_blocks(cal_ctx* c, int64_t n, int64_t ld, int nb, const std::vector<double*>& dQ, const int* widths,
                   int m, double* dX, bool doreorth, std::vector<std::vector<double>>& R);
// projectAndNormalize.m:3-90 against several blocks (general path; X kept).
int project_and_normalize_blocks_dev(cal_ctx* c, int64_t n, int64_t ld, int nblocks, const std::vector<double*>& dQ,
                                     const int* widths, int m, const double* dX, bool doreorth, double* dY,
                                     const PanelOut& Qout, std::vector<std::vector<double>>& RZ, double* R,
                                     bool* reorth, int* rank);
// Q factor of a wide (m > 16) block by CholQR2 (+ shifted pass).
int normalize_wide_dev(cal_ctx* c, int64_t n, int64_t ld, const double* dX, int m, double* dQ, double* dW);
// Halo exchange of a column (distributed only; no-op for one rank).
int halo_exchange(cal_ctx* c, double* x);
// y = A x (with modes), handling the halo first.  Mode 3 (CSR only):
// y = A (x / sqrt(*xnrm)), xnrm a device scalar.
int spmv_dev(cal_ctx* c, const double* x, double* y, int mode, double shift, double im2,
             const double* xprev, const double* xnrm = nullptr);
// y = A x (mode 0, or 3 on CSR) on stream st without timers or statistics
// (one rank; the asynchronous normest)
hipError_t spmv_on_stream(const cal_ctx* c, const double* x, double* y, int mode, const double* xnrm, hipStream_t st);
int allreduce_sum(cal_ctx* c, double* d_buf, int64_t count);
// d_recv[p * count + i] = rank p's d_send[i] (in rank order, every rank)
int allgather(cal_ctx* c, const double* d_send, double* d_recv, int64_t count);

// Householder TSQR of Z (tsqr.m:7-12): Z = W (direct, dM null, W.total = m)
// or Z = W * M (dM: W.total x m column-major on the device, formed per row),
// optionally followed by Z += W(:, 0:w2) * M2 on the rounded W * M (dM2).
// Q -> Qout (n x m), R -> host (m x m, diag >= 0, the reference's sign fix).
// Multi-GPU: the tree's root is taken over all ranks (allgather + redundant
// top levels).  Runs c->pre_wait before its one host wait.  m <= 32.
int tsqr_dev(cal_ctx* c, int64_t n, const Panel& W, const double* dM, int m, const PanelOut& Qout, double* R,
             const double* dM2 = nullptr, int w2 = 0);
bool tsqr_ok(int m);
// whether normalize / projectAndNormalize use TSQR here (tier1: a host-pointer call)
bool use_tsqr(const cal_ctx* c, int m, bool tier1);

}  // namespace cal
