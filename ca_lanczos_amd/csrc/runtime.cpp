// runtime.cpp -- context lifecycle, device buffers, matrix upload, timers.
#include <algorithm>
#include <cmath>
#include <thread>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <unordered_map>
#include <string>
#include <vector>

#include "cal_internal.hpp"
#include "comm.hpp"

namespace cal {

constexpr int kRowBlockRows = 256;   // rows per CSR-stream block (= threads)
constexpr int kRowBlockNnz = 2048;   // nonzeros staged in LDS per block

// A library-owned worker thread (the host-staged overlap schedule's comm
// thread) points this at its own string, so it never writes the context's
// error state concurrently with the caller's thread; the caller moves the
// message into the context after the join.
static thread_local std::string* tl_err_sink = nullptr;

int set_error(cal_ctx* c, int code, const std::string& msg) {
    if (tl_err_sink) *tl_err_sink = msg;
    else if (c) c->err = msg;
    return code;
}

int hip_fail(cal_ctx* c, hipError_t e, const char* what) {
    std::string m = std::string("HIP error '") + hipGetErrorString(e) + "' in " + what;
    return set_error(c, CAL_ERR_HIP, m);
}

hipError_t scratch_malloc(void** p, size_t bytes) {
    hipError_t e = hipMalloc(p, bytes);
#ifdef CAL_TEST_HOOKS
    if (e == hipSuccess) e = hipMemset(*p, 0xFF, bytes);
    if (e == hipSuccess) e = hipDeviceSynchronize();
#endif
    return e;
}

static int grow(cal_ctx* c, double** p, size_t* cap, size_t need) {
    if (need <= *cap) return 0;
    if (*p) CAL_HIP(c, hipFree(*p));
    *p = nullptr;
    // by half again at least: a Gram that widens every outer iteration ('full',
    // 'selective', the restarts) reallocates O(log) times, not every other step
    // (each reallocation synchronises the device and allocates: 0.3-0.5 ms)
    size_t n = std::max({need, *cap + *cap / 2, (size_t)4096});
    CAL_HIP(c, scratch_malloc((void**)p, n * sizeof(double)));
    *cap = n;
    return 0;
}

int ensure_partial(cal_ctx* c, size_t doubles) { return grow(c, &c->d_partial, &c->partial_cap, doubles); }
int ensure_scratch(cal_ctx* c, size_t doubles) { return grow(c, &c->d_scratch, &c->scratch_cap, doubles); }

int ensure_small(cal_ctx* c, size_t doubles) {
    if (doubles <= c->small_cap) return 0;
    if (c->d_small) CAL_HIP(c, hipFree(c->d_small));
    if (c->h_small) CAL_HIP(c, hipHostFree(c->h_small));
    c->d_small = nullptr;
    c->h_small = nullptr;
    size_t n = std::max(doubles, (size_t)65536);
    CAL_HIP(c, scratch_malloc((void**)&c->d_small, n * sizeof(double)));
    CAL_HIP(c, hipHostMalloc((void**)&c->h_small, n * sizeof(double), hipHostMallocDefault));
    c->small_cap = n;
    return 0;
}

int ensure_red(cal_ctx* c, size_t doubles) {
    if (doubles <= c->red_cap) return 0;
    if (c->d_red) CAL_HIP(c, hipFree(c->d_red));
    if (c->h_red) CAL_HIP(c, hipHostFree(c->h_red));
    c->d_red = nullptr;
    c->h_red = nullptr;
    size_t n = std::max(doubles, (size_t)65536);
    CAL_HIP(c, scratch_malloc((void**)&c->d_red, n * sizeof(double)));
    CAL_HIP(c, hipHostMalloc((void**)&c->h_red, n * sizeof(double), hipHostMallocDefault));
    c->red_cap = n;
    return 0;
}

int ensure_pub(cal_ctx* c) {
    if (c->h_pub) return 0;
    // coherent (uncached), mapped: GPU stores reach host memory directly
    CAL_HIP(c, hipHostMalloc((void**)&c->h_pub, kPubDoubles * sizeof(double),
                             hipHostMallocMapped | hipHostMallocCoherent));
    std::fill(c->h_pub, c->h_pub + kPubDoubles, 0.0);
    CAL_HIP(c, hipHostGetDevicePointer((void**)&c->d_pub, c->h_pub, 0));
    c->pub_seq = 0;
    return 0;
}

int ensure_work(cal_ctx* c, int cols, int64_t ld) {
    if (cols <= c->work_cols && ld == c->work_ld) return 0;
    // grow by half again (the Ritz diagnostics ask for s more columns every
    // outer iteration; each reallocation frees, i.e. synchronises, and zeroes)
    int alloc = cols;
    if (ld == c->work_ld) alloc = std::max(cols, c->work_cols + c->work_cols / 2);
    alloc = (alloc + 15) & ~15;
    if (c->d_work) CAL_HIP(c, hipFree(c->d_work));
    c->d_work = nullptr;
    c->work_cols = 0;
    CAL_HIP(c, hipMalloc((void**)&c->d_work, (size_t)alloc * ld * sizeof(double)));
    CAL_HIP(c, hipMemsetAsync(c->d_work, 0, (size_t)alloc * ld * sizeof(double), c->stream));
    c->work_cols = alloc;
    c->work_ld = ld;
    return 0;
}

double* work_col(cal_ctx* c, int j) { return c->d_work + (size_t)j * c->work_ld; }

int timer_begin(cal_ctx* c, int kind, double bytes) {
    if (!c->timing) return -1;
    CalTimerRec r;
    r.kind = kind;
    r.bytes = bytes;
    if (c->event_pool.size() >= 2) {
        r.a = c->event_pool.back();
        c->event_pool.pop_back();
        r.b = c->event_pool.back();
        c->event_pool.pop_back();
    } else {
        // timing-only events: no system-scope fence at record, so the pair
        // does not write back and invalidate the caches around the kernel it
        // brackets (with the default fence a bracketed Gram sweep read 6 %
        // above its rocprof duration); readers synchronise first
        if (hipEventCreateWithFlags(&r.a, hipEventDisableSystemFence) != hipSuccess) return -1;
        if (hipEventCreateWithFlags(&r.b, hipEventDisableSystemFence) != hipSuccess) return -1;
    }
    hipEventRecord(r.a, c->stream);
    c->timers.push_back(r);
    return (int)c->timers.size() - 1;
}

void timer_end(cal_ctx* c, int idx) {
    if (idx < 0) return;
    hipEventRecord(c->timers[idx].b, c->stream);
}

int timer_begin_on(cal_ctx* c, int kind, hipStream_t st) {
    const hipStream_t saved = c->stream;
    c->stream = st;
    const int t = timer_begin(c, kind);
    c->stream = saved;
    return t;
}

void timer_end_on(cal_ctx* c, int idx, hipStream_t st) {
    if (idx < 0) return;
    hipEventRecord(c->timers[idx].b, st);
}

// Split rows into CSR-stream blocks: <= kRowBlockRows rows and <= kRowBlockNnz
// nonzeros; a longer row gets a block of its own (long-row path).
static void build_row_blocks(int64_t n, const std::vector<int>& rowptr, std::vector<int>& blk, int* max_nnz) {
    blk.clear();
    blk.push_back(0);
    int64_t r = 0;
    int mx = 0;
    while (r < n) {
        const int64_t start = r;
        const int len0 = rowptr[r + 1] - rowptr[r];
        if (len0 > kRowBlockNnz) {
            r++;
            blk.push_back((int)r);
            continue;
        }
        int nz = 0;
        while (r < n && r - start < kRowBlockRows) {
            const int len = rowptr[r + 1] - rowptr[r];
            if (len > kRowBlockNnz || nz + len > kRowBlockNnz) break;
            nz += len;
            r++;
        }
        mx = std::max(mx, nz);
        blk.push_back((int)r);
    }
    *max_nnz = mx;
}

static void free_matrix(cal_ctx* c) {
    DevMatrix& A = c->A;
    if (A.rowptr) hipFree(A.rowptr);
    if (A.col) hipFree(A.col);
    if (A.val) hipFree(A.val);
    if (A.blk) hipFree(A.blk);
    if (A.send_idx) hipFree(A.send_idx);
    if (A.send_buf) hipFree(A.send_buf);
    if (A.pat) hipFree(A.pat);
    if (A.pinfo) hipFree(A.pinfo);
    if (A.pdelta) hipFree(A.pdelta);
    if (A.pval) hipFree(A.pval);
    if (A.ppat) hipFree(A.ppat);
    if (A.ppinfo) hipFree(A.ppinfo);
    if (A.ppoff) hipFree(A.ppoff);
    if (A.ppval) hipFree(A.ppval);
    if (A.rzval) hipFree(A.rzval);
    if (A.rzmask) hipFree(A.rzmask);
    if (A.rowkey8) hipFree(A.rowkey8);
    if (A.rowmask) hipFree(A.rowmask);
    if (A.wavemask) hipFree(A.wavemask);
    A = DevMatrix();
    if (c->d_work) hipFree(c->d_work);
    c->d_work = nullptr;
    c->work_cols = 0;
    c->has_A = false;
}

// ---- row-pattern analysis -------------------------------------------------
constexpr int kMaxPatterns = 65535;
constexpr int kMaxPatternEntries = 1 << 16;
constexpr int kMaxPatternLen = 32;

// Returns false when the matrix has too many distinct rows for the format.
// n stored rows; stored row r is local row r - org (col is local-origin relative).
static bool build_patterns(int64_t n, int64_t org, const std::vector<int>& rowptr, const std::vector<int>& col,
                           const double* val, std::vector<uint16_t>& pat, std::vector<int2>& pinfo,
                           std::vector<int>& pdelta, std::vector<double>& pval, int* maxlen) {
    pat.assign(n, 0);
    pinfo.clear();
    pdelta.assign(1, 0);  // entry 0: sentinel (delta 0) for empty rows
    pval.assign(1, 0.0);
    std::unordered_map<uint64_t, std::vector<int>> buckets;
    int mx = 0;
    for (int64_t r = 0; r < n; ++r) {
        const int p0 = rowptr[r], len = rowptr[r + 1] - p0;
        if (len > kMaxPatternLen) return false;
        mx = std::max(mx, len);
        uint64_t h = 1469598103934665603ull ^ (uint64_t)len;
        for (int j = 0; j < len; ++j) {
            uint64_t vb;
            std::memcpy(&vb, &val[p0 + j], 8);
            const uint64_t d = (uint64_t)(uint32_t)(col[p0 + j] - (int)(r - org));
            h = (h ^ d) * 1099511628211ull;
            h = (h ^ vb) * 1099511628211ull;
        }
        auto& cand = buckets[h];
        int found = -1;
        for (int id : cand) {
            const int2 pi = pinfo[id];
            if (pi.y != len) continue;
            bool same = true;
            for (int j = 0; j < len && same; ++j)
                same = pdelta[pi.x + j] == col[p0 + j] - (int)(r - org) &&
                       std::memcmp(&pval[pi.x + j], &val[p0 + j], 8) == 0;
            if (same) {
                found = id;
                break;
            }
        }
        if (found < 0) {
            if ((int)pinfo.size() >= kMaxPatterns) return false;
            if ((int)pdelta.size() + len > kMaxPatternEntries) return false;
            found = (int)pinfo.size();
            pinfo.push_back(make_int2(len > 0 ? (int)pdelta.size() : 0, len));
            for (int j = 0; j < len; ++j) {
                pdelta.push_back(col[p0 + j] - (int)(r - org));
                pval.push_back(val[p0 + j]);
            }
            cand.push_back(found);
        }
        pat[r] = (uint16_t)found;
    }
    *maxlen = mx;
    return true;
}

// Pair patterns: rows 2t and 2t+1 get one merged pattern over the union O of
// their column offsets, so one 16-B load x[r+o .. r+o+1] per entry serves
// both rows.  Entry flags say which row uses it; each row still adds its own
// entries in column order (bit-identical).  A merged entry loads the
// unused half too, so that half must be a valid vector entry: a local row
// or an index some row references (received halo).  Pairs that fail this,
// and the lone last row of an odd n, are marked kPairSplit (per-row path).
constexpr int kMaxPairLen = 16;

static bool build_pair_patterns(int64_t n, int64_t org, const std::vector<uint16_t>& pat,
                                const std::vector<int2>& pinfo,
                                const std::vector<int>& pdelta, const std::vector<double>& pval,
                                const std::vector<int>& col, std::vector<uint16_t>& ppat, std::vector<int2>& ppinfo,
                                std::vector<int>& ppoff, std::vector<double>& ppval, int* pmaxlen, bool* pcanon,
                                int* slots) {
    int64_t cmin = -org, cmax = n - 1 - org;  // local coordinates
    for (int v : col) {
        cmin = std::min<int64_t>(cmin, v);
        cmax = std::max<int64_t>(cmax, v);
    }
    std::vector<uint8_t> ref((size_t)(cmax - cmin + 1), 0);
    for (int v : col) ref[(size_t)(v - cmin)] = 1;
    auto valid = [&](int64_t i) {  // i: local coordinate
        return (i >= -org && i < n - org) || (i >= cmin && i <= cmax && ref[(size_t)(i - cmin)]);
    };
    struct Merged {
        int id;
        std::vector<int> pad0, pad1;  // offsets row 2t / 2t+1 loads without using
    };
    // Canonical slots: when the matrix has few distinct offsets overall, every
    // pair pattern lists all of them in one global order (unused slots load
    // x[r..r+1], flags 0), so the lanes of a wave load the same offset in
    // the same slot even across pattern changes (fewer cache lines per load).
    std::vector<int> U;
    for (size_t e = 1; e < pdelta.size(); ++e) U.push_back(pdelta[e]);
    std::sort(U.begin(), U.end());
    U.erase(std::unique(U.begin(), U.end()), U.end());
    const bool canonical = !U.empty() && (int)U.size() <= 8;
    *pcanon = canonical;
    for (size_t k = 0; canonical && k < U.size(); ++k) slots[k] = U[k];
    std::unordered_map<uint32_t, Merged> seen;
    const int64_t npairs = (n + 1) / 2;
    ppat.assign(npairs, (uint16_t)kPairSplit);
    ppinfo.clear();
    ppoff.clear();
    ppval.clear();
    int mx = 0;
    for (int64_t t = 0; t < npairs; ++t) {
        const int64_t r = 2 * t;
        if (r + 1 >= n) break;  // lone last row: split
        const int p0 = pat[r], p1 = pat[r + 1];
        const uint32_t key = ((uint32_t)p0 << 16) | (uint32_t)p1;
        auto it = seen.find(key);
        if (it == seen.end()) {
            const int2 a = pinfo[p0], b = pinfo[p1];
            std::vector<int> O;
            for (int e = 0; e < a.y; ++e) O.push_back(pdelta[a.x + e]);
            for (int e = 0; e < b.y; ++e) O.push_back(pdelta[b.x + e]);
            std::sort(O.begin(), O.end());
            O.erase(std::unique(O.begin(), O.end()), O.end());
            if (canonical) O = U;
            if ((int)O.size() > kMaxPairLen || (int)ppinfo.size() >= kPairSplit) return false;
            Merged mg;
            mg.id = (int)ppinfo.size();
            ppinfo.push_back(make_int2((int)ppoff.size(), (int)O.size()));
            for (int o : O) {
                if (o >= (1 << 28) || o <= -(1 << 28)) return false;
                int f = 0;
                double v0 = 0.0, v1 = 0.0;
                for (int e = 0; e < a.y; ++e)
                    if (pdelta[a.x + e] == o) {
                        f |= 1;
                        v0 = pval[a.x + e];
                    }
                for (int e = 0; e < b.y; ++e)
                    if (pdelta[b.x + e] == o) {
                        f |= 2;
                        v1 = pval[b.x + e];
                    }
                if (f == 0) {  // canonical slot unused by both rows: load x[r..r+1]
                    ppoff.push_back(0);
                    ppval.push_back(0.0);
                    ppval.push_back(0.0);
                    continue;
                }
                if (!(f & 1)) mg.pad0.push_back(o);
                if (!(f & 2)) mg.pad1.push_back(o);
                ppoff.push_back(o * 4 + f);
                ppval.push_back(v0);
                ppval.push_back(v1);
            }
            mx = std::max(mx, (int)O.size());
            it = seen.emplace(key, std::move(mg)).first;
        }
        bool ok = true;
        for (int o : it->second.pad0) ok = ok && valid(r - org + o);
        for (int o : it->second.pad1) ok = ok && valid(r - org + 1 + o);
        if (ok) ppat[t] = (uint16_t)it->second.id;
    }
    *pmaxlen = mx;
    return !ppinfo.empty();
}

// Upload a local matrix: n_rows stored rows, the n_local local ones from
// stored row ext_off.  col: local column ids relative to the local origin
// (negative ids address the left halo); lpad / rext: halo extent on either
// side of the local rows in every vector column.
int upload_matrix(cal_ctx* c, int64_t n_rows, int64_t ext_off, int64_t n_local, int64_t n_global, int64_t row0,
                  int64_t nghost, int64_t lpad, int64_t rext, const std::vector<int>& rowptr,
                  const std::vector<int>& col, const double* val) {
    free_matrix(c);
    DevMatrix& A = c->A;
    A.n_local = n_local;
    A.n_rows = n_rows;
    A.ext_off = ext_off;
    A.n_global = n_global;
    A.row0 = row0;
    A.nghost = nghost;
    A.nnz = rowptr[n_rows];
    A.nnz_loc = rowptr[ext_off + n_local] - rowptr[ext_off];
    A.lpad = ((lpad + 63) / 64) * 64;
    // two rows of slack past the data: the plane march reads row pairs up
    // to n + 1 (planes_ok needs ld >= n + 2; with n a multiple of 64 the
    // row-pair kernel ran instead: lap2d_1000 5905-6022 -> 6112-6234
    // outer-it/s with the slack, profiles/r05/ld_slack/)
    A.ld = ((A.lpad + n_local + rext + 2 + 63) / 64) * 64;
    if (A.ld == 0) A.ld = 64;
    // storage format: row patterns when the table is small (auto) or forced
    if (c->spmv_format != 1) {
        std::vector<uint16_t> pat;
        std::vector<int2> pinfo;
        std::vector<int> pdelta;
        std::vector<double> pval;
        int mx = 0;
        const bool ok = n_rows > 0 && build_patterns(n_rows, ext_off, rowptr, col, val, pat, pinfo, pdelta, pval, &mx);
        if (ok) {
            A.use_pat = true;
            A.npat = (int)pinfo.size();
            A.nent = (int)pdelta.size();
            A.maxlen = mx <= 8 ? std::max(mx, 1) : (mx <= 16 ? 16 : 32);
            // 8 zero bytes past the ids: the plane march's aligned dword key loads
            CAL_HIP(c, hipMalloc((void**)&A.pat, n_rows * sizeof(uint16_t) + 8));
            CAL_HIP(c, hipMemset(A.pat, 0, n_rows * sizeof(uint16_t) + 8));
            CAL_HIP(c, hipMalloc((void**)&A.pinfo, pinfo.size() * sizeof(int2)));
            CAL_HIP(c, hipMalloc((void**)&A.pdelta, pdelta.size() * sizeof(int)));
            CAL_HIP(c, hipMalloc((void**)&A.pval, pval.size() * sizeof(double)));
            CAL_HIP(c, hipMemcpy(A.pat, pat.data(), n_rows * sizeof(uint16_t), hipMemcpyHostToDevice));
            CAL_HIP(c, hipMemcpy(A.pinfo, pinfo.data(), pinfo.size() * sizeof(int2), hipMemcpyHostToDevice));
            CAL_HIP(c, hipMemcpy(A.pdelta, pdelta.data(), pdelta.size() * sizeof(int), hipMemcpyHostToDevice));
            CAL_HIP(c, hipMemcpy(A.pval, pval.data(), pval.size() * sizeof(double), hipMemcpyHostToDevice));
            std::vector<uint16_t> ppat;
            std::vector<int2> ppinfo;
            std::vector<int> ppoff;
            std::vector<double> ppval;
            int pmx = 0;
            bool canon = false;
            if (build_pair_patterns(n_rows, ext_off, pat, pinfo, pdelta, pval, col, ppat, ppinfo, ppoff, ppval, &pmx,
                                    &canon, A.pslot)) {
                A.use_pair = true;
                A.nppat = (int)ppinfo.size();
                A.npent = (int)ppoff.size();
                A.pmaxlen = pmx <= 8 ? std::max(pmx, 1) : 16;
                A.pcanon = canon && A.pmaxlen == pmx;
                A.npsplit = std::count(ppat.begin(), ppat.end(), (uint16_t)kPairSplit);
                CAL_HIP(c, hipMalloc((void**)&A.ppat, ppat.size() * sizeof(uint16_t)));
                CAL_HIP(c, hipMalloc((void**)&A.ppinfo, ppinfo.size() * sizeof(int2)));
                CAL_HIP(c, hipMalloc((void**)&A.ppoff, ppoff.size() * sizeof(int)));
                CAL_HIP(c, hipMalloc((void**)&A.ppval, ppval.size() * sizeof(double)));
                CAL_HIP(c, hipMemcpy(A.ppat, ppat.data(), ppat.size() * sizeof(uint16_t), hipMemcpyHostToDevice));
                CAL_HIP(c, hipMemcpy(A.ppinfo, ppinfo.data(), ppinfo.size() * sizeof(int2), hipMemcpyHostToDevice));
                CAL_HIP(c, hipMemcpy(A.ppoff, ppoff.data(), ppoff.size() * sizeof(int), hipMemcpyHostToDevice));
                CAL_HIP(c, hipMemcpy(A.ppval, ppval.data(), ppval.size() * sizeof(double), hipMemcpyHostToDevice));
                // the plane march (k_resid_planes): a single slab without halos whose
                // canonical slots include -P and +P (the largest offset) and whose
                // other slots reach H <= 256 rows: lap3d (P = N^2, H = N + 1) and
                // lap2d (P = N, H = 2) qualify
                const int L = A.pmaxlen;
                if (A.pcanon && L >= 2 && ext_off == 0 && n_rows == n_local && A.lpad == 0 &&
                    A.pslot[L - 1] >= 256 && A.pslot[0] == -A.pslot[L - 1] && (size_t)A.npat * L <= 2048) {
                    int H = 0;
                    for (int e = 1; e < L - 1; ++e) H = std::max(H, std::abs(A.pslot[e]));
                    H = (H + 1) & ~1;
                    if (H <= 256) {
                        std::vector<double> rz((size_t)A.npat * L, 0.0);
                        std::vector<uint8_t> rm((size_t)A.npat, 0);
                        for (int q = 0; q < A.npat; ++q)
                            for (int e = 0; e < pinfo[q].y; ++e) {
                                const int o = pdelta[pinfo[q].x + e];
                                for (int k = 0; k < L; ++k)
                                    if (A.pslot[k] == o) {
                                        rz[(size_t)q * L + k] = pval[pinfo[q].x + e];
                                        rm[q] |= (uint8_t)(1u << k);
                                    }
                            }
                        CAL_HIP(c, hipMalloc((void**)&A.rzval, rz.size() * sizeof(double)));
                        CAL_HIP(c, hipMemcpy(A.rzval, rz.data(), rz.size() * sizeof(double), hipMemcpyHostToDevice));
                        CAL_HIP(c, hipMalloc((void**)&A.rzmask, rm.size()));
                        CAL_HIP(c, hipMemcpy(A.rzmask, rm.data(), rm.size(), hipMemcpyHostToDevice));
                        // uniform slot values: one value per slot over every pattern that has it
                        bool uni = true;
                        for (int k = 0; k < L && uni; ++k) {
                            bool seen = false;
                            for (int q = 0; q < A.npat && uni; ++q)
                                if (rm[q] >> k & 1u) {
                                    const double v = rz[(size_t)q * L + k];
                                    if (!seen) A.cval[k] = v;
                                    else uni = std::memcmp(&v, &A.cval[k], 8) == 0;
                                    seen = true;
                                }
                        }
                        if (uni) {  // 1-B mask keys (8 zero bytes past the rows: dword key loads)
                            std::vector<uint8_t> km((size_t)n_rows + 8, 0);
                            for (int64_t r = 0; r < n_rows; ++r) km[(size_t)r] = rm[pat[(size_t)r]];
                            CAL_HIP(c, hipMalloc((void**)&A.rowmask, km.size()));
                            CAL_HIP(c, hipMemcpy(A.rowmask, km.data(), km.size(), hipMemcpyHostToDevice));
                            A.cuniform = true;
                        } else if (A.npat <= 256) {  // 1-B keys (8 zero bytes past the rows: dword key loads)
                            std::vector<uint8_t> k8((size_t)n_rows + 8, 0);
                            for (int64_t r = 0; r < n_rows; ++r) k8[(size_t)r] = (uint8_t)pat[(size_t)r];
                            CAL_HIP(c, hipMalloc((void**)&A.rowkey8, k8.size()));
                            CAL_HIP(c, hipMemcpy(A.rowkey8, k8.data(), k8.size(), hipMemcpyHostToDevice));
                        }
                        A.plane_P = A.pslot[L - 1];
                        A.plane_H = H;
                        // the waves' missing-slot masks (cal_internal.hpp DevMatrix::wavemask)
                        {
                            const int64_t P = A.plane_P;
                            const int64_t nxy = (P + kPlaneBlockRows - 1) / kPlaneBlockRows;
                            const int64_t nz = (n_rows + P - 1) / P;
                            const unsigned full = (1u << L) - 1u;
                            std::vector<uint32_t> wm((size_t)(nz + 1) * nxy, 0u);
                            for (int64_t z = 0; z < nz; ++z)
                                for (int64_t b = 0; b < nxy; ++b) {
                                    uint32_t v = 0;
                                    for (int w = 0; w < 4; ++w) {
                                        unsigned m = 0;
                                        const int64_t r0 = z * P + b * kPlaneBlockRows + 128 * w;
                                        for (int64_t r = r0; r < r0 + 128; ++r)
                                            m |= r < n_rows ? full & ~(unsigned)rm[pat[(size_t)r]] : full;
                                        v |= (uint32_t)m << (8 * w);
                                    }
                                    wm[(size_t)(z * nxy + b)] = v;
                                }
                            CAL_HIP(c, hipMalloc((void**)&A.wavemask, wm.size() * sizeof(uint32_t)));
                            CAL_HIP(c, hipMemcpy(A.wavemask, wm.data(), wm.size() * sizeof(uint32_t),
                                                 hipMemcpyHostToDevice));
                        }
                    }
                }
            }
        } else if (c->spmv_format == 2) {
            return set_error(c, CAL_ERR_UNSUPPORTED, "row-pattern format requested but the matrix has too many "
                                                     "distinct rows (or rows longer than 32)");
        }
    }
    // CSR-stream row blocks over the local rows (the CSR path never runs on
    // an extended matrix: the mpk requires the row-pattern format)
    std::vector<int> blk;
    int max_nnz = 0;
    std::vector<int> rp_loc(rowptr.begin() + ext_off, rowptr.begin() + ext_off + n_local + 1);
    build_row_blocks(n_local, rp_loc, blk, &max_nnz);
    A.nblk = (int)blk.size() - 1;
    int nit = (max_nnz + 255) / 256;
    if (nit < 1) nit = 1;
    if (nit > 8) nit = 8;
    A.nit = nit;
    CAL_HIP(c, hipMalloc((void**)&A.rowptr, (n_rows + 1) * sizeof(int)));
    CAL_HIP(c, hipMalloc((void**)&A.col, std::max<int64_t>(A.nnz, 1) * sizeof(int)));
    CAL_HIP(c, hipMalloc((void**)&A.val, std::max<int64_t>(A.nnz, 1) * sizeof(double)));
    CAL_HIP(c, hipMalloc((void**)&A.blk, blk.size() * sizeof(int)));
    CAL_HIP(c, hipMemcpy(A.rowptr, rowptr.data(), (n_rows + 1) * sizeof(int), hipMemcpyHostToDevice));
    if (A.nnz > 0) {
        CAL_HIP(c, hipMemcpy(A.col, col.data(), A.nnz * sizeof(int), hipMemcpyHostToDevice));
        CAL_HIP(c, hipMemcpy(A.val, val, A.nnz * sizeof(double), hipMemcpyHostToDevice));
    }
    CAL_HIP(c, hipMemcpy(A.blk, blk.data(), blk.size() * sizeof(int), hipMemcpyHostToDevice));
    c->has_A = true;
    c->A_gen++;
    return 0;
}

static PatArgs pat_args(const DevMatrix& A, int64_t o, int64_t len, const double* x, double* y, int mode,
                        double shift, double im2, const double* xprev) {
    const int64_t d = o - A.ext_off;  // launch origin relative to the local origin
    PatArgs p;
    p.pat = A.pat + o;
    p.pinfo = A.pinfo;
    p.pdelta = A.pdelta;
    p.pval = A.pval;
    p.n = len;
    p.nblk = (int)((len + 255) / 256);
    p.x = x + d;
    p.y = y + d;
    p.xprev = xprev ? xprev + d : nullptr;
    p.shift = shift;
    p.im2 = im2;
    p.mode = mode;
    p.maxlen = A.maxlen;
    p.npat = A.npat;
    p.nent = A.nent;
    p.ppat = A.use_pair ? A.ppat + o / 2 : nullptr;
    p.ppinfo = A.ppinfo;
    p.ppoff = A.ppoff;
    p.ppval = A.ppval;
    p.nppat = A.nppat;
    p.npent = A.npent;
    p.pmaxlen = A.pmaxlen;
    p.pcanon = A.pcanon ? 1 : 0;
    for (int k = 0; k < 8; ++k) p.pslot[k] = A.pslot[k];
    {
        // the +-1 slots from the neighbouring lanes (k_spmv_pair*)
        const int z = A.pmaxlen / 2;
        p.pmid = (A.pcanon && (A.pmaxlen & 1) && A.pmaxlen >= 3 && A.pslot[z] == 0 &&
                  A.pslot[z - 1] == -1 && A.pslot[z + 1] == 1)
                     ? z
                     : -1;
    }
    p.xlo = -(A.lpad + d);
    p.xhi = A.ld - (A.lpad + d);
    p.ld = A.ld;
    if (A.rzval && o == A.ext_off && len == A.n_local) {
        p.rzval = A.rzval;
        p.rzmask = A.rzmask;
        p.rowkey8 = A.rowkey8;
        p.rowmask = A.rowmask;
        p.wavemask = A.wavemask;
        p.cuniform = A.cuniform ? 1 : 0;
        for (int k = 0; k < 8; ++k) p.cval[k] = A.cval[k];
        p.plane_P = A.plane_P;
        p.plane_H = A.plane_H;
    }
    return p;
}

// algorithmic bytes of a row-pattern SpMV over len rows: the key (1 B per row
// with pair patterns / the plane march's keys, 2 B otherwise), x, y, and
// the previous power for MODE 2
static double pat_spmv_bytes(const DevMatrix& A, int64_t len, int mode) {
    return (double)len * ((A.use_pair ? 1 : 2) + 16 + (mode == 2 ? 8 : 0));
}

int spmv_range(cal_ctx* c, int64_t o, int64_t len, const double* x, double* y, int mode, double shift, double im2,
               const double* xprev) {
    const DevMatrix& A = c->A;
    if (o < 0 || (o & 1) || len < 0 || o + len > A.n_rows)
        return set_error(c, CAL_ERR_ARG, "spmv_range: bad stored-row range");
    const PatArgs p = pat_args(A, o, len, x, y, mode, shift, im2, xprev);
    c->stat_spmv_rows += len;
    const int t = timer_begin(c, 0, pat_spmv_bytes(A, len, mode));
    CAL_HIP(c, launch_spmv_pat(p, c->stream));
    timer_end(c, t);
    return 0;
}

// y = A x on stream st, no timer and no statistics: the asynchronous normest
// (lanczos.cpp) on its own stream beside the solver's.  One rank (no halo).
// Mode 0, or 3 on CSR (y = A (x / sqrt(*xnrm))).
hipError_t spmv_on_stream(const cal_ctx* c, const double* x, double* y, int mode, const double* xnrm, hipStream_t st) {
    const DevMatrix& A = c->A;
    if (mode != 0 && mode != 3) return hipErrorInvalidValue;
    if (A.use_pat) {
        if (mode != 0) return hipErrorInvalidValue;
        return launch_spmv_pat(pat_args(A, A.ext_off, A.n_local, x, y, 0, 0.0, 0.0, nullptr), st);
    }
    SpmvArgs a;
    a.rowptr = A.rowptr;
    a.col = A.col;
    a.val = A.val;
    a.blk = A.blk;
    a.nblk = A.nblk;
    a.x = x;
    a.y = y;
    a.xprev = nullptr;
    a.shift = 0.0;
    a.im2 = 0.0;
    a.xnrm = xnrm;
    a.mode = mode | (A.nit << 8);
    a.nt = (int64_t)12 * A.nnz > ((int64_t)256 << 20) ? 1 : 0;
    return launch_spmv(a, st);
}

int spmv_resid_pair_blocks(cal_ctx* c) {
    const DevMatrix& A = c->A;
    if (!c->has_A || !A.use_pat || !A.use_pair) return 0;
    // alignment is that of the work columns (16-B aligned origins)
    const PatArgs p = pat_args(A, A.ext_off, A.n_local, nullptr, nullptr, 1, 0.0, 0.0, nullptr);
    return spmv_pair_resid_blocks(p);
}

int spmv_resid_pair_dev(cal_ctx* c, const double* x, double lr, double* partial, int* blocks) {
    const DevMatrix& A = c->A;
    *blocks = 0;
    if (!c->has_A || !A.use_pat || !A.use_pair) return 0;
    const PatArgs p = pat_args(A, A.ext_off, A.n_local, x, nullptr, 1, lr, 0.0, nullptr);
    const int nb = spmv_pair_resid_blocks(p);
    if (nb <= 0) return 0;
    const int t = timer_begin(c, 3);
    CAL_HIP(c, launch_spmv_pair_resid(p, lr, partial, c->stream));
    timer_end(c, t);
    *blocks = nb;
    return 0;
}

int spmv_resid_pair_multi_blocks(cal_ctx* c) {
    const DevMatrix& A = c->A;
    if (!c->has_A || !A.use_pat || !A.use_pair) return 0;
    const PatArgs p = pat_args(A, A.ext_off, A.n_local, nullptr, nullptr, 1, 0.0, 0.0, nullptr);
    return spmv_pair_resid_multi_blocks(p);
}

int spmv_resid_pair_multi_dev(cal_ctx* c, const double* X, int64_t ldx, const int* col, const double* lam,
                              const int* out, int npr, double* partial, int64_t pstride) {
    const DevMatrix& A = c->A;
    if (!c->has_A || !A.use_pat || !A.use_pair) return set_error(c, CAL_ERR_ARG, "pair residuals: no pair patterns");
    const PatArgs p = pat_args(A, A.ext_off, A.n_local, X, nullptr, 1, 0.0, 0.0, nullptr);
    CAL_HIP(c, launch_spmv_pair_resid_multi(p, X, ldx, col, lam, out, npr, partial, pstride, c->stream));
    return 0;
}

// Two stored-row ranges [o1, o1 + len1) and [o2, o2 + len2) in one launch
// (the pair kernel skips the gap; the row kernels take two launches).
int spmv_range2(cal_ctx* c, int64_t o1, int64_t len1, int64_t o2, int64_t len2, const double* x, double* y, int mode,
                double shift, double im2, const double* xprev) {
    const DevMatrix& A = c->A;
    if (len1 == 0) return spmv_range(c, o2, len2, x, y, mode, shift, im2, xprev);
    if (len2 == 0) return spmv_range(c, o1, len1, x, y, mode, shift, im2, xprev);
    if (o1 < 0 || (o1 & 1) || (len1 & 1) || (o2 & 1) || len2 < 0 || o2 < o1 + len1 || o2 + len2 > A.n_rows)
        return set_error(c, CAL_ERR_ARG, "spmv_range2: bad stored-row ranges");
    PatArgs p = pat_args(A, o1, len1 + len2, x, y, mode, shift, im2, xprev);
    p.gap_at = len1 / 2;
    p.gap = (o2 - o1) / 2 - p.gap_at;
    c->stat_spmv_rows += len1 + len2;
    const int t = timer_begin(c, 0, pat_spmv_bytes(A, len1 + len2, mode));
    CAL_HIP(c, launch_spmv_pat(p, c->stream));
    timer_end(c, t);
    return 0;
}

int spmv_dev(cal_ctx* c, const double* x, double* y, int mode, double shift, double im2, const double* xprev,
             const double* xnrm) {
    if (!c->has_A) return set_error(c, CAL_ERR_NOMATRIX, "no matrix set on the context");
    if (mode == 3 && (c->A.use_pat || !xnrm)) return set_error(c, CAL_ERR_ARG, "spmv_dev: mode 3 needs CSR and xnrm");
    CAL_TRY(halo_exchange(c, const_cast<double*>(x)));
    if (c->A.use_pat) return spmv_range(c, c->A.ext_off, c->A.n_local, x, y, mode, shift, im2, xprev);
    SpmvArgs a;
    a.xnrm = xnrm;
    a.rowptr = c->A.rowptr;
    a.col = c->A.col;
    a.val = c->A.val;
    a.blk = c->A.blk;
    a.nblk = c->A.nblk;
    a.x = x;
    a.y = y;
    a.xprev = xprev;
    a.shift = shift;
    a.im2 = im2;
    a.mode = mode | (c->A.nit << 8);
    // col + val of the stored rows against the 256 MB Infinity Cache
    a.nt = (int64_t)12 * c->A.nnz > ((int64_t)256 << 20) ? 1 : 0;
    c->stat_spmv_rows += c->A.n_local;
    // 12 nnz + 20 n + 4 (+ 8 n for the previous power, MODE 2)
    const int t = timer_begin(c, 0, 12.0 * c->A.nnz + 20.0 * c->A.n_local + 4.0 + (mode == 2 ? 8.0 * c->A.n_local : 0.0));
    CAL_HIP(c, launch_spmv(a, c->stream));
    timer_end(c, t);
    return 0;
}

// CA matrix powers: after one halo exchange of q's s-deep
// ghost zone, power j (1-based) is valid on global rows [row0 - (s-j) bl,
// row1 + (s-j) br) -- it reads power j-1 one band further out -- so power s
// is the local slab.  Each range is launched as a sub-range of the stored
// rows, its start rounded down to even (the pair kernel's alignment) and its
// length up to even: the extra edge rows are computed from stale halo data
// and never read by a valid row of the next power (they lie one row outside
// its reach), and masked loads keep them from leaking into their pair rows.
//
// Overlap (RCCL): the exchange runs on the communicator's stream while the
// compute stream works through the interior trapezoid -- power j on
// [row0 + j bl, row1 - j br), which reads only power j-1's interior and, for
// j = 1, q's own rows.  The boundary pieces [glo_j, row0 + j bl) and
// [row1 - j br, ghi_j) follow the exchange, both sides in one launch, after
// every interior power: they read the boundary of power j-1 and the interior
// next to it.  A boundary launch recomputes at most one interior edge row
// (the even rounding) from valid data, so its bits do not change; the
// interior launch's own extra edge row is stale until that boundary launch
// overwrites it and is outside the next interior power's reach.
struct PowRange {
    int64_t o, len;  // stored rows, o even
};

static PowRange stored_range(const DevMatrix& A, int64_t glo, int64_t ghi) {
    int64_t o = glo - A.row0 + A.ext_off;
    const int64_t e = ghi - A.row0 + A.ext_off;
    o &= ~(int64_t)1;
    int64_t len = std::max<int64_t>(0, e - o);
    if ((len & 1) && o + len < A.n_rows) ++len;
    return {o, len};
}

// 0 off, 1 on (default for RCCL), from CAL_MPK_OVERLAP; CAL_MPK_FAKE_BAND=b
// splits a single rank's powers the same way with band b (launch-cost and
// two-range-kernel checks: no exchange is involved, the bits are unchanged)
static int mpk_overlap_env() {
    const char* e = std::getenv("CAL_MPK_OVERLAP");
    return e ? std::atoi(e) : -1;
}
static int64_t mpk_fake_band() {
    const char* e = std::getenv("CAL_MPK_FAKE_BAND");
    return e ? (int64_t)std::atoll(e) : (int64_t)0;
}

int powers_dev(cal_ctx* c, int s, const double* q, double* const* Y, const double* shift, const double* im2,
               const double* const* xprev) {
    const DevMatrix& A = c->A;
    c->powers_launches = s;  // one SpMV-class launch per power
    auto mode_of = [&](int j) { return shift ? ((im2 && im2[j] != 0.0) ? 2 : 1) : 0; };
    auto launch = [&](int j, const PowRange& r1, const PowRange& r2) {  // power j (1-based)
        return spmv_range2(c, r1.o, r1.len, r2.o, r2.len, j == 1 ? q : Y[j - 2], Y[j - 1], mode_of(j - 1),
                           shift ? shift[j - 1] : 0.0, im2 ? im2[j - 1] : 0.0, xprev ? xprev[j - 1] : nullptr);
    };
    const int64_t row1 = A.row0 + A.n_local;
    const bool mpk = A.mpk && A.use_pat && s <= A.mpk_depth && s > 1;
    const int64_t fake = (!mpk && !A.mpk && A.use_pat && s > 1 && A.nghost == 0) ? mpk_fake_band() : 0;
    if (!mpk && fake <= 0) {
        c->powers_schedule = 0;
        for (int j = 0; j < s; ++j)
            CAL_TRY(spmv_dev(c, j == 0 ? q : Y[j - 1], Y[j], mode_of(j), shift ? shift[j] : 0.0,
                             im2 ? im2[j] : 0.0, xprev ? xprev[j] : nullptr));
        return 0;
    }
    // global rows of power j and whether each side waits for the exchange
    const int64_t bl = mpk ? A.band_l : fake, br = mpk ? A.band_r : fake;
    auto glo = [&](int j) { return mpk ? std::max(A.ext_lo, A.row0 - (int64_t)(s - j) * bl) : A.row0; };
    auto ghi = [&](int j) { return mpk ? std::min(A.ext_hi, row1 + (int64_t)(s - j) * br) : row1; };
    const bool dep_lo = mpk ? A.ext_lo < A.row0 : true, dep_hi = mpk ? A.ext_hi > row1 : true;
    auto ilo = [&](int j) { return dep_lo ? A.row0 + (int64_t)j * bl : glo(j); };
    auto ihi = [&](int j) { return dep_hi ? row1 - (int64_t)j * br : ghi(j); };
    Comm* m = c->comm;
    const bool comm_stream = mpk && m && m->stream && m->ev_q && m->ev_halo;
    const bool rccl = comm_stream && m->kind == 1;
    const int ov = mpk_overlap_env();
    const bool split = (fake > 0 || (mpk && (ov == 1 || (ov < 0 && rccl)))) && (dep_lo || dep_hi) &&
                       ilo(s) + 4 < ihi(s);
    c->powers_schedule = split ? (rccl ? 2 : (comm_stream ? 4 : 3)) : 1;
    if (!split) {
        CAL_TRY(halo_exchange_deep(c, const_cast<double*>(q), s, c->stream));
        for (int j = 1; j <= s; ++j) CAL_TRY(launch(j, stored_range(A, glo(j), ghi(j)), PowRange{0, 0}));
        return 0;
    }
    // The exchange runs on the communicator's stream behind an event recorded
    // when q is ready; the compute stream waits for ev_halo only before the
    // boundary pieces.  RCCL enqueues its send/recv kernels there directly.
    // The host-staged twin (schedule 4) keeps the same event graph: a comm
    // thread waits for ev_q through the stream, stages q's pieces to the host,
    // runs the exchange callbacks, copies the ghost rows back on the same
    // stream and records ev_halo, while this thread enqueues the interior
    // powers; the wait on ev_halo is enqueued after the join (an event must be
    // recorded before a stream can wait for it).
    std::thread comm_thread;
    int comm_status = 0;
    std::string comm_err;
    if (comm_stream) {
        CAL_HIP(c, hipEventRecord(m->ev_q, c->stream));
        CAL_HIP(c, hipStreamWaitEvent(m->stream, m->ev_q, 0));
        if (rccl) {
            CAL_TRY(halo_exchange_deep(c, const_cast<double*>(q), s, m->stream));
            CAL_HIP(c, hipEventRecord(m->ev_halo, m->stream));
        } else {
            comm_thread = std::thread([c, m, q, s, &comm_status, &comm_err]() {
                tl_err_sink = &comm_err;
                hipSetDevice(c->device);
                comm_status = halo_exchange_deep(c, const_cast<double*>(q), s, m->stream);
                if (comm_status == 0 && hipEventRecord(m->ev_halo, m->stream) != hipSuccess)
                    comm_status = set_error(c, CAL_ERR_HIP, "halo event record");
                tl_err_sink = nullptr;
            });
        }
    } else if (mpk) {
        CAL_TRY(halo_exchange_deep(c, const_cast<double*>(q), s, c->stream));
    }
    int interior_status = 0;
    for (int j = 1; j <= s && interior_status == 0; ++j)
        interior_status = launch(j, stored_range(A, ilo(j), ihi(j)), PowRange{0, 0});
    if (comm_thread.joinable()) comm_thread.join();
    CAL_TRY(interior_status);
    if (comm_status != 0) return set_error(c, comm_status, comm_err);
    if (comm_stream) CAL_HIP(c, hipStreamWaitEvent(c->stream, m->ev_halo, 0));
    for (int j = 1; j <= s; ++j) {
        const PowRange lo = dep_lo ? stored_range(A, glo(j), ilo(j)) : PowRange{0, 0};
        const PowRange hi = dep_hi ? stored_range(A, ihi(j), ghi(j)) : PowRange{0, 0};
        if (lo.len > 0 && hi.len > 0 && hi.o < lo.o + lo.len)
            return set_error(c, CAL_ERR_ARG, "powers_dev: boundary ranges overlap");
        CAL_TRY(launch(j, lo, hi));
    }
    return 0;
}

}  // namespace cal

using namespace cal;

extern "C" {

int cal_version(void) { return 1; }

int cal_device_count(int* count) {
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    if (e != hipSuccess) n = 0;
    if (count) *count = n;
    return e == hipSuccess ? 0 : CAL_ERR_HIP;
}

int cal_create(int device, cal_ctx** out) {
    if (!out) return CAL_ERR_ARG;
    *out = nullptr;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return CAL_ERR_HIP;
    if (device < 0 || device >= n) return CAL_ERR_ARG;
    if (hipSetDevice(device) != hipSuccess) return CAL_ERR_HIP;
    cal_ctx* c = new cal_ctx();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return CAL_ERR_HIP;
    }
    *out = c;
    return 0;
}

void cal_lanczos_free_state(cal_ctx* c);  // lanczos.cpp

void cal_destroy(cal_ctx* c) {
    if (!c) return;
    hipSetDevice(c->device);
    hipStreamSynchronize(c->stream);
    if (c->nest_stream) hipStreamSynchronize(c->nest_stream);
    cal_lanczos_free_state(c);
    cal::comm_destroy(c);
    free_matrix(c);
    if (c->d_partial) hipFree(c->d_partial);
    if (c->d_red) hipFree(c->d_red);
    if (c->h_red) hipHostFree(c->h_red);
    if (c->d_small) hipFree(c->d_small);
    if (c->h_small) hipHostFree(c->h_small);
    if (c->d_scratch) hipFree(c->d_scratch);
    for (auto& r : c->timers) {
        hipEventDestroy(r.a);
        hipEventDestroy(r.b);
    }
    for (auto e : c->event_pool) hipEventDestroy(e);
    if (c->orth_event) hipEventDestroy(c->orth_event);
    if (c->d_tsqr) hipFree(c->d_tsqr);
    if (c->d_zbuf) hipFree(c->d_zbuf);
    if (c->d_tsqrv) hipFree(c->d_tsqrv);
    if (c->d_fold) hipFree(c->d_fold);
    if (c->pbw.d) hipFree(c->pbw.d);
    if (c->pbw.h) hipHostFree(c->pbw.h);
    if (c->pbw.ev) hipEventDestroy(c->pbw.ev);
    if (c->h_pub) hipHostFree(c->h_pub);
    if (c->aux_stream) hipStreamDestroy(c->aux_stream);
    for (hipGraphExec_t& g : c->nest_exec)
        if (g) hipGraphExecDestroy(g);
    if (c->d_nest) hipFree(c->d_nest);
    if (c->h_nest) hipHostFree(c->h_nest);
    if (c->nest_event) hipEventDestroy(c->nest_event);
    if (c->nest_stream) hipStreamDestroy(c->nest_stream);

    hipStreamDestroy(c->stream);
    delete c;
}

const char* cal_last_error(const cal_ctx* c) { return c ? c->err.c_str() : "null context"; }

int cal_synchronize(cal_ctx* c) {
    if (!c) return CAL_ERR_ARG;
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    return 0;
}

int cal_timer_enable(cal_ctx* c, int on) {
    if (!c) return CAL_ERR_ARG;
    c->timing = on != 0;
    return 0;
}

int cal_timer_reset(cal_ctx* c) {
    if (!c) return CAL_ERR_ARG;
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    for (auto& r : c->timers) {
        c->event_pool.push_back(r.a);
        c->event_pool.push_back(r.b);
    }
    c->timers.clear();
    return 0;
}

int cal_timer_bytes(cal_ctx* c, const char* kind, double* bytes) {
    if (!c || !kind || !bytes) return CAL_ERR_ARG;
    int k = -1;
    if (!strcmp(kind, "spmv")) k = 0;
    else if (!strcmp(kind, "gram")) k = 1;
    else if (!strcmp(kind, "apply")) k = 2;
    else if (!strcmp(kind, "other")) k = 3;
    else if (!strcmp(kind, "allreduce")) k = 4;
    else if (!strcmp(kind, "halo")) k = 5;
    else if (!strcmp(kind, "normest")) k = 6;
    else if (strcmp(kind, "all")) return set_error(c, CAL_ERR_ARG, "unknown timer kind");
    double b = 0.0;
    for (auto& r : c->timers)
        if (k < 0 || r.kind == k) b += r.bytes;
    *bytes = b;
    return 0;
}

int cal_timer_read(cal_ctx* c, const char* kind, int64_t* count, double* total_ms) {
    if (!c || !kind) return CAL_ERR_ARG;
    int k = -1;
    if (!strcmp(kind, "spmv")) k = 0;
    else if (!strcmp(kind, "gram")) k = 1;
    else if (!strcmp(kind, "apply")) k = 2;
    else if (!strcmp(kind, "other")) k = 3;
    else if (!strcmp(kind, "allreduce")) k = 4;
    else if (!strcmp(kind, "halo")) k = 5;
    else if (!strcmp(kind, "normest")) k = 6;
    else if (strcmp(kind, "all")) return set_error(c, CAL_ERR_ARG, "unknown timer kind");
    CAL_HIP(c, hipStreamSynchronize(c->stream));
    int64_t cnt = 0;
    double tot = 0.0;
    for (auto& r : c->timers) {
        if (k >= 0 && r.kind != k) continue;
        float ms = 0.f;
        CAL_HIP(c, hipEventSynchronize(r.b));  // timers on the communicator's stream too
        CAL_HIP(c, hipEventElapsedTime(&ms, r.a, r.b));
        cnt++;
        tot += ms;
    }
    if (count) *count = cnt;
    if (total_ms) *total_ms = tot;
    return 0;
}

int cal_set_matrix_csr(cal_ctx* c, int64_t n, const int64_t* rowptr, const int32_t* colind, const double* val) {
    if (!c || n < 0 || !rowptr || (n > 0 && rowptr[n] > 0 && (!colind || !val)))
        return set_error(c, CAL_ERR_ARG, "cal_set_matrix_csr: bad arguments");
    if (c->comm && c->comm->nranks > 1)
        return set_error(c, CAL_ERR_ARG, "distributed context: use cal_set_matrix_csr_dist");
    const int64_t nnz = rowptr[n];
    if (nnz >= ((int64_t)1 << 31) || n >= ((int64_t)1 << 31))
        return set_error(c, CAL_ERR_UNSUPPORTED, "n and nnz must be < 2^31 per rank");
    hipSetDevice(c->device);
    std::vector<int> rp(n + 1), col(nnz);
    for (int64_t i = 0; i <= n; ++i) rp[i] = (int)rowptr[i];
    for (int64_t p = 0; p < nnz; ++p) {
        const int32_t j = colind[p];
        if (j < 0 || j >= n) return set_error(c, CAL_ERR_ARG, "column index out of range");
        col[p] = j;
    }
    for (int64_t i = 0; i < n; ++i)
        if (rp[i + 1] < rp[i]) return set_error(c, CAL_ERR_ARG, "row pointers must be non-decreasing");
    return upload_matrix(c, n, 0, n, n, 0, 0, 0, 0, rp, col, val);
}

int cal_set_matrix_csc(cal_ctx* c, int64_t n, const int64_t* jc, const int64_t* ir, const double* pr) {
    // MATLAB's CSC (mwIndex jc/ir) transposed into CSR by a counting sort over
    // the rows, so the device holds A, not A', whatever its symmetry: SpMV.m:8
    // is a general A*v.  Walking the columns in order leaves every CSR row with
    // ascending column indices, which is MATLAB's own accumulation order for
    // y(i) in sparse mtimes (column by column), so y is bit-identical to A*v.
    // For a symmetric A the result equals the CSC arrays read as CSR.
    if (!c || n < 0 || !jc) return set_error(c, CAL_ERR_ARG, "cal_set_matrix_csc: bad arguments");
    if (n >= ((int64_t)1 << 31)) return set_error(c, CAL_ERR_UNSUPPORTED, "n and nnz must be < 2^31 per rank");
    if (jc[0] != 0) return set_error(c, CAL_ERR_ARG, "column pointers must start at 0");
    for (int64_t j = 0; j < n; ++j)
        if (jc[j + 1] < jc[j]) return set_error(c, CAL_ERR_ARG, "column pointers must be non-decreasing");
    const int64_t nnz = jc[n];
    if (nnz >= ((int64_t)1 << 31)) return set_error(c, CAL_ERR_UNSUPPORTED, "n and nnz must be < 2^31 per rank");
    if (nnz > 0 && (!ir || !pr)) return set_error(c, CAL_ERR_ARG, "cal_set_matrix_csc: bad arguments");
    std::vector<int64_t> rowptr(n + 1, 0);
    for (int64_t p = 0; p < nnz; ++p) {
        if (ir[p] < 0 || ir[p] >= n) return set_error(c, CAL_ERR_ARG, "row index out of range");
        rowptr[ir[p] + 1]++;
    }
    for (int64_t i = 0; i < n; ++i) rowptr[i + 1] += rowptr[i];
    std::vector<int64_t> next(rowptr.begin(), rowptr.end() - 1);
    std::vector<int32_t> col32(nnz);
    std::vector<double> val(nnz);
    for (int64_t j = 0; j < n; ++j)
        for (int64_t p = jc[j]; p < jc[j + 1]; ++p) {
            const int64_t q = next[ir[p]]++;
            col32[q] = (int32_t)j;
            val[q] = pr[p];
        }
    return cal_set_matrix_csr(c, n, rowptr.data(), col32.data(), val.data());
}

int cal_set_spmv_format(cal_ctx* c, const char* fmt) {
    if (!c || !fmt) return CAL_ERR_ARG;
    if (!strcmp(fmt, "auto")) c->spmv_format = 0;
    else if (!strcmp(fmt, "csr")) c->spmv_format = 1;
    else if (!strcmp(fmt, "pattern")) c->spmv_format = 2;
    else return set_error(c, CAL_ERR_ARG, "spmv format must be auto, csr or pattern");
    return 0;
}

int cal_set_orth_coef(cal_ctx* c, const char* where) {
    if (!c || !where) return CAL_ERR_ARG;
    if (!strcmp(where, "device")) c->orth_coef_device = true;
    else if (!strcmp(where, "host")) c->orth_coef_device = false;
    else return set_error(c, CAL_ERR_ARG, "orth coefficients: \"device\" or \"host\"");
    return 0;
}

int cal_spmv_pair_info(cal_ctx* c, int* npairpatterns, int* nentries, int64_t* nsplit) {
    if (!c) return CAL_ERR_ARG;
    if (!c->has_A) return set_error(c, CAL_ERR_NOMATRIX, "no matrix set on the context");
    if (npairpatterns) *npairpatterns = c->A.use_pair ? c->A.nppat : 0;
    if (nentries) *nentries = c->A.use_pair ? c->A.npent : 0;
    if (nsplit) *nsplit = c->A.use_pair ? c->A.npsplit : 0;
    return 0;
}

int cal_spmv_plane_info(cal_ctx* c, int64_t* plane_P, int* plane_H, int* key_mode) {
    if (!c) return CAL_ERR_ARG;
    if (!c->has_A) return set_error(c, CAL_ERR_NOMATRIX, "no matrix set on the context");
    const bool on = c->A.use_pair && c->A.plane_P > 0;
    if (plane_P) *plane_P = on ? c->A.plane_P : 0;
    if (plane_H) *plane_H = on ? c->A.plane_H : 0;
    if (key_mode) *key_mode = !on ? -1 : (c->A.cuniform ? 0 : (c->A.npat <= 256 ? 1 : 2));
    return 0;
}

int cal_spmv_format(cal_ctx* c, int* is_pattern, int* npatterns, int* nentries) {
    if (!c) return CAL_ERR_ARG;
    if (!c->has_A) return set_error(c, CAL_ERR_NOMATRIX, "no matrix set on the context");
    if (is_pattern) *is_pattern = c->A.use_pat ? 1 : 0;
    if (npatterns) *npatterns = c->A.npat;
    if (nentries) *nentries = c->A.nent;
    return 0;
}

int cal_set_mpk_depth(cal_ctx* c, int depth) {
    if (!c || depth < 1 || depth > 64) return set_error(c, CAL_ERR_ARG, "mpk depth must be in 1..64");
    c->mpk_depth_req = depth;
    return 0;
}

int cal_mpk_info(cal_ctx* c, int* depth, int64_t* band_l, int64_t* band_r, int64_t* n_rows) {
    if (!c) return CAL_ERR_ARG;
    if (!c->has_A) return set_error(c, CAL_ERR_NOMATRIX, "no matrix set on the context");
    if (depth) *depth = c->A.mpk ? c->A.mpk_depth : 1;
    if (band_l) *band_l = c->A.band_l;
    if (band_r) *band_r = c->A.band_r;
    if (n_rows) *n_rows = c->A.n_rows;
    return 0;
}

int cal_set_normalize(cal_ctx* c, const char* kind) {
    if (!c || !kind) return CAL_ERR_ARG;
    std::string k(kind);
    for (auto& ch : k) ch = (char)tolower(ch);
    if (k == "auto") c->normalize_kind = 0;
    else if (k == "tsqr") c->normalize_kind = 1;
    else if (k == "cholqr2") c->normalize_kind = 2;
    else return set_error(c, CAL_ERR_ARG, "normalize backend must be auto, tsqr or cholqr2");
    return 0;
}

int cal_get_normalize(cal_ctx* c, int* kind) {
    if (!c || !kind) return CAL_ERR_ARG;
    *kind = c->normalize_kind;
    return 0;
}

int cal_tsqr_fold_stats(cal_ctx* c, long long* runs, long long* declined, double* last_est) {
    if (!c) return CAL_ERR_ARG;
    if (runs) *runs = c->fold_runs;
    if (declined) *declined = c->fold_declined;
    if (last_est) *last_est = c->fold_last_est;
    return 0;
}

int cal_set_tsqr_fold_tol(cal_ctx* c, double tol) {
    if (!c) return CAL_ERR_ARG;
    if (std::isnan(tol)) return set_error(c, CAL_ERR_ARG, "cal_set_tsqr_fold_tol: tol is NaN");
    // only lowering it keeps the orthogonality guarantee (more declines, each
    // redone on the explicit-Z path); a larger tol would accept folds whose
    // loss-of-orthogonality estimate the default declines
    if (tol > kFoldTol)
        return set_error(c, CAL_ERR_ARG, "cal_set_tsqr_fold_tol: tol above the default 1e-14 would weaken the "
                                         "orthogonality guarantee");
    c->fold_tol = tol;
    return 0;
}

int cal_mpk_schedule(cal_ctx* c, int* schedule) {
    if (!c || !schedule) return CAL_ERR_ARG;
    *schedule = c->powers_schedule;
    return 0;
}

int cal_powers_launches(cal_ctx* c, int* launches) {
    if (!c || !launches) return CAL_ERR_ARG;
    *launches = c->powers_launches;
    return 0;
}

int cal_matrix_info(cal_ctx* c, int64_t* n_local, int64_t* nnz_local, int64_t* n_global, int64_t* nghost) {
    if (!c) return CAL_ERR_ARG;
    if (!c->has_A) return set_error(c, CAL_ERR_NOMATRIX, "no matrix set on the context");
    if (n_local) *n_local = c->A.n_local;
    if (nnz_local) *nnz_local = c->A.nnz_loc;
    if (n_global) *n_global = c->A.n_global;
    if (nghost) *nghost = c->A.nghost;
    return 0;
}

}  // extern "C"
