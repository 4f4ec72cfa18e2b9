// kernels_plan.hip -- per-block erasure-decode planning on the GPU.
//
// RS (RS8 and RS16): the reference builds a k x k decoding matrix whose erased source
// rows are replaced by the generator rows of the first surviving parities and inverts it
// by Gauss-Jordan (src/common/normEncoderRS8.cpp:656-725, 766-889).  Only the rows of
// the erased symbols are ever used (:727-756) and, with D = [[A, B], [0, I]] in
// (erased, rest) order, those rows of D^-1 are [A^-1, A^-1 B].  So the repair is
//     z_t = parity(P_t) ^ sum_{c present} G[P_t][c] * d_c      (stage 1: gather rows of G)
//     d_E = A^-1 z,   A[t][s] = G[P_t][E_s]                      (stage 2: e x e inverse)
// which is byte-identical (the inverse is unique) and needs only an e x e inversion per
// block instead of k x k.  One wavefront plans one block: parity selection follows the
// reference's ascending scan (:660-718), the e x [A | I] Gauss-Jordan runs lane-parallel
// over columns in LDS.
//
// MDP: the reference decode (src/common/normEncoderMDP.cpp:333-430) is linear in the
// surviving vectors; the plan evaluates its syndrome / erasure-locator / Omega / Forney
// chain symbolically into one coefficient per (erased source symbol, surviving vector):
//   C[r][v] = Dinv_r * gamma_v * sum_{l<m} (gamma_v beta_r)^l Lambda_{m-1-l}(beta_r)
// with gamma_v = alpha^(nvecs-1-v), beta_r = alpha^((255-k_r) % 255), Lambda_u the prefix
// sums of the locator evaluated at beta_r and Dinv_r = GINV[lambda'(beta_r)] (GINV[0]=1).
#include "nfec_internal.hpp"

namespace nfec {

namespace {

constexpr int kWave = 64;
constexpr uint32_t kPlanLdsMaxE = 64;
constexpr uint32_t kPlanLrowMaxE = 256;  // log-domain elimination up to this e

__device__ __forceinline__ uint32_t uni(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }

template <typename E>
struct FieldDev {
    const E* exp;          // 2q entries
    const uint16_t* log;   // q+1 entries, log[0] = q
    uint32_t q;
    __device__ __forceinline__ uint32_t mul(uint32_t a, uint32_t b) const
    {
        return (a && b) ? (uint32_t)exp[(uint32_t)log[a] + (uint32_t)log[b]] : 0u;
    }
    __device__ __forceinline__ uint32_t inv(uint32_t a) const
    {
        return a <= 1 ? a : (uint32_t)exp[q - (uint32_t)log[a]];
    }
};

template <typename E>
__global__ __launch_bounds__(kWave) void rs_plan_kernel(RsPlanArgs a)
{
    __shared__ E lds_work[kPlanLdsMaxE * 2 * kPlanLdsMaxE];
    __shared__ uint16_t lds_E[256], lds_P[256];
    __shared__ E lds_fac[256];
    __shared__ uint8_t lds_exp8[512];
    __shared__ uint16_t lds_log8[256];
    __shared__ uint16_t lds_lrow[2 * kPlanLrowMaxE];  // log of the normalised pivot row (q: zero)

    const uint32_t lane = threadIdx.x;
    const uint32_t b = blockIdx.x;
    FieldDev<E> f;
    f.q = sizeof(E) == 1 ? 255u : 65535u;
    if constexpr (sizeof(E) == 1) {
        const uint8_t* ge = reinterpret_cast<const uint8_t*>(a.exp_tab);
        for (uint32_t i = lane; i < 510; i += kWave) lds_exp8[i] = ge[i];
        for (uint32_t i = lane; i < 256; i += kWave) lds_log8[i] = a.log_tab[i];
        __syncthreads();
        f.exp = reinterpret_cast<const E*>(lds_exp8);
        f.log = lds_log8;
    } else {
        f.exp = reinterpret_cast<const E*>(a.exp_tab);
        f.log = a.log_tab;
    }

    const uint32_t k = a.k, m = a.m;
    const uint32_t nd = a.num_data ? uni(a.num_data[b]) : k;
    const uint32_t ec = uni(a.erasure_counts[b]);
    const uint16_t* locs = a.erasure_locs + (uint64_t)b * a.erasure_stride;
    int32_t status = (int32_t)ec;

    // ---- validate and split erasures (sorted: source first, then parity) ----
    bool ok = nd >= 1 && nd <= k && ec <= a.erasure_stride && ec <= m;
    uint32_t es = 0;
    if (ok) {
        for (uint32_t i = 0; i < ec; ++i) {
            const uint32_t l = locs[i];
            if (l >= nd + m || (i > 0 && l <= locs[i - 1])) ok = false;
            if (l < nd) ++es;
        }
    }
    if (!ok) status = 0;
    // erased / substitute-parity lists and pivot factors: LDS up to 256 erasures, else the
    // block's global scratch after its e x 2e matrix
    const uint32_t cs = a.coef_stride;
    uint8_t* wb = a.work ? reinterpret_cast<uint8_t*>(a.work) + (uint64_t)b * a.work_block_bytes : nullptr;
    const bool big = es > 256;
    if (ok && big && (!wb || es > cs)) { ok = false; status = 0; }  // workspace not sized for it
    uint16_t* listE = big ? reinterpret_cast<uint16_t*>(wb + (uint64_t)cs * 2 * cs * sizeof(E)) : lds_E;
    uint16_t* listP = big ? listE + cs : lds_P;
    E* fac = big ? reinterpret_cast<E*>(listP + cs) : lds_fac;
    if (ok && es > 0) {
        // surviving parities in ascending slot order (reference scan :660-718)
        if (lane == 0) {
            uint32_t next = es, np = 0;
            for (uint32_t s = nd; s < nd + m && np < es; ++s) {
                if (next < ec && locs[next] == s) { ++next; continue; }
                listP[np++] = (uint16_t)s;
            }
            for (uint32_t i = 0; i < es; ++i) listE[i] = locs[i];
            if (np < es) listP[0] = 0xffff;  // not enough parity
        }
        __syncthreads();
        if (listP[0] == 0xffff) { ok = false; status = 0; }
    }
    const uint32_t e = ok ? es : 0;
    // stage 1 by encode: the substitute parities are rows 0..e-1 (listP ascending from nd)
    const bool by_encode = a.rows1 && e > 0 && nd == k && listP[e - 1] == nd + e - 1;
    if (lane == 0) {
        if (a.status) a.status[b] = status;
        a.rows[b] = (int32_t)e;
        a.cols2[b] = (uint16_t)e;
        if (a.rows1) a.rows1[b] = by_encode ? 0 : (int32_t)e;
    }
    if (e == 0) return;

    // ---- stage-1 gather matrix and slots ----
    const E* gp = reinterpret_cast<const E*>(a.gen_parity);
    for (uint32_t c = lane; c < nd && !by_encode; c += kWave) {
        E* coef1 = reinterpret_cast<E*>(a.coef1) + (uint64_t)b * k * cs;
        uint16_t* islots = a.in_slots1 + (uint64_t)b * k;
        // is c erased? (E sorted: binary search)
        int32_t s_idx = -1;
        {
            uint32_t lo = 0, hi = e;  // first index with listE[i] >= c
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (listE[mid] < c) lo = mid + 1;
                else hi = mid;
            }
            if (lo < e && listE[lo] == c) s_idx = (int32_t)lo;
        }
        islots[c] = s_idx >= 0 ? listP[s_idx] : (uint16_t)c;
        for (uint32_t t = 0; t < cs; ++t) {
            E v = 0;
            if (t < e) {
                if (s_idx >= 0) v = (E)((uint32_t)s_idx == t);
                else v = gp[(uint64_t)(listP[t] - nd) * k + c];
            }
            coef1[(uint64_t)c * cs + t] = v;
        }
    }

    // ---- stage 2: invert A[t][s] = G[P_t][E_s] via Gauss-Jordan on [A | I] ----
    const uint32_t w2 = 2 * e;
    E* work = e <= kPlanLdsMaxE ? lds_work : reinterpret_cast<E*>(wb);
    for (uint32_t idx = lane; idx < e * w2; idx += kWave) {
        const uint32_t t = idx / w2, col = idx % w2;
        E v;
        if (col < e) v = gp[(uint64_t)(listP[t] - nd) * k + listE[col]];
        else v = (E)(col - e == t);
        work[idx] = v;
    }
    __syncthreads();
    bool singular = false;
    for (uint32_t j = 0; j < e; ++j) {
        // pivot: first row >= j with a non-zero entry in column j
        uint32_t piv = 0xffffffffu;
        for (uint32_t base = j; base < e; base += kWave) {
            const uint32_t r = base + lane;
            const bool nz = r < e && work[r * w2 + j] != 0;
            const uint64_t mask = __ballot(nz);
            if (mask) {
                piv = base + (uint32_t)__ffsll((unsigned long long)mask) - 1;
                break;
            }
        }
        if (piv == 0xffffffffu) { singular = true; break; }
        if (piv != j) {
            for (uint32_t col = lane; col < w2; col += kWave) {
                E tmp = work[j * w2 + col];
                work[j * w2 + col] = work[piv * w2 + col];
                work[piv * w2 + col] = tmp;
            }
            __syncthreads();
        }
        if (e <= kPlanLrowMaxE) {
            // log domain: the normalised pivot row and the factors are turned into logs once
            // per pivot, so each eliminated entry costs one exp-table read instead of two log
            // reads and an exp read (for GF(2^16) these are L2 gathers)
            const uint32_t q = f.q;
            const uint32_t lpinv = (q - (uint32_t)f.log[work[j * w2 + j]]) % q;
            for (uint32_t col = lane; col < w2; col += kWave) {
                const uint32_t v = work[j * w2 + col];
                const uint32_t lv = v ? ((uint32_t)f.log[v] + lpinv) % q : q;
                lds_lrow[col] = (uint16_t)lv;
                work[j * w2 + col] = v ? f.exp[lv] : (E)0;
            }
            // factors: column j of the other rows (not touched by the normalisation)
            for (uint32_t r = lane; r < e; r += kWave)
                if (r != j) fac[r] = (E)f.log[work[r * w2 + j]];  // log 0 = q: no update
            __syncthreads();
            for (uint32_t idx = lane; idx < e * w2; idx += kWave) {
                const uint32_t r = idx / w2, col = idx % w2;
                if (r == j) continue;
                const uint32_t lf = fac[r], lc = lds_lrow[col];
                if (lf != q && lc != q) work[idx] ^= f.exp[lf + lc];
            }
            __syncthreads();
        } else {
            const uint32_t pinv = f.inv(work[j * w2 + j]);
            for (uint32_t col = lane; col < w2; col += kWave) work[j * w2 + col] = (E)f.mul(pinv, work[j * w2 + col]);
            __syncthreads();
            // snapshot column j (the elimination factors) before any row is updated
            for (uint32_t r = lane; r < e; r += kWave) fac[r] = work[r * w2 + j];
            __syncthreads();
            for (uint32_t idx = lane; idx < e * w2; idx += kWave) {
                const uint32_t r = idx / w2, col = idx % w2;
                if (r == j) continue;
                const uint32_t factor = fac[r];
                if (factor) work[idx] ^= (E)f.mul(factor, work[j * w2 + col]);
            }
            __syncthreads();
        }
    }
    if (singular) {
        if (lane == 0) {
            if (a.status) a.status[b] = 0;
            a.rows[b] = 0;
            a.cols2[b] = 0;
        }
        return;
    }
    E* coef2 = reinterpret_cast<E*>(a.coef2) + (uint64_t)b * cs * cs;
    for (uint32_t idx = lane; idx < cs * cs; idx += kWave) {
        const uint32_t t = idx / cs, s = idx % cs;  // column t (input z_t), row s (output)
        E v = 0;
        if (t < e && s < e) v = work[s * w2 + e + t];
        coef2[idx] = v;
    }
    uint16_t* oslots = a.out_slots2 + (uint64_t)b * k;
    for (uint32_t s = lane; s < e; s += kWave) oslots[s] = listE[s];
    if (by_encode) {
        // the stage-1 encode reads every source slot: the erased ones must read as zero
        if (lane == 0) atomicMax(a.rmax, e);
        uint8_t* blk = a.zero_base + (uint64_t)b * a.zero_block_stride;
        const uint32_t words = a.zero_vec >> 3;
        for (uint32_t s = 0; s < e; ++s) {
            uint2* p = reinterpret_cast<uint2*>(blk + (uint64_t)listE[s] * a.zero_seg_stride);
            for (uint32_t w = lane; w < words; w += kWave) p[w] = make_uint2(0u, 0u);
        }
    }
}


// ---------------------------------------------------------------------------------
// RS16 plan in closed form: the outputs of rs_plan_kernel<uint16_t> (status, rows, the stage-1
// gather matrix or the by-encode marking, the erased slots) with A^-1 from the Cauchy form of
// the Lagrange generator instead of Gauss-Jordan (the same algebra as rs_plan2_kernel; the
// inverse is unique, so the coefficients are identical):
//     A^-1[s][t] = exp(lA[s] + lB[t] - log(x_s ^ y_t))
//     lA[s] = log W'(x_s) + sum_t log(x_s ^ y_t) - sum_{s' != s} log(x_s ^ x_s')
//     lB[t] = -log W(y_t) + sum_s log(y_t ^ x_s) - sum_{t' != t} log(y_t ^ y_t')
// O(e^2) table terms per block instead of O(e^3).  One wavefront per block, e <= kPlanCfMaxE;
// the GF(2^16) log / exp tables are read through L2.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kWave) void rs16_plan_cf_kernel(RsPlanArgs a)
{
    __shared__ uint16_t listE[kPlanCfMaxE], listP[kPlanCfMaxE];
    __shared__ uint16_t xs[kPlanCfMaxE], yt[kPlanCfMaxE];
    __shared__ int32_t lA[kPlanCfMaxE], lB[kPlanCfMaxE];
    __shared__ uint32_t np_s;
    // lost parity rows as a bitmap and the stage-2 column -> substitute index map, for the
    // usual sizes (ec, ncol <= kPlanCfScan); past them the serial scan / binary search below
    constexpr uint32_t kPlanCfScan = 1024;
    __shared__ uint32_t pbits[kPlanCfScan / 32];
    __shared__ int16_t pinv[kPlanCfScan];
    // e <= 64: the e x e logs lg[x_s ^ y_t] kept in LDS (each gathered once for the row sums of
    // lA, the column sums of lB and the inverse's entries), the x-x and y-y log sums gathered
    // for s < s' only (symmetric).  The kernel is bound by these random gathers through the
    // vector memory path (~one cache line per lane).
    constexpr uint32_t kPlanCfSmall = 64, kLxyStride = kPlanCfSmall + 1;
    __shared__ uint16_t Lxy[kPlanCfSmall * kLxyStride];
    __shared__ int32_t xxs[kPlanCfSmall], yys[kPlanCfSmall];
    const uint32_t lane = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint16_t* ex = reinterpret_cast<const uint16_t*>(a.exp_tab);  // 2q entries
    const uint16_t* lg = a.log_tab;                                      // lg[0] = q
    constexpr int32_t q = 65535;
    const uint32_t k = a.k, m = a.m;
    const uint32_t nd = a.num_data ? uni(a.num_data[b]) : k;
    const uint32_t ec = uni(a.erasure_counts[b]);
    const uint16_t* locs = a.erasure_locs + (uint64_t)b * a.erasure_stride;
    int32_t status = (int32_t)ec;

    // ---- validate (lane-parallel: sorted, in range) and count source erasures ----
    bool ok = nd >= 1 && nd <= k && ec <= a.erasure_stride && ec <= m;
    uint32_t es = 0;
    if (ok) {
        bool bad = false;
        uint32_t nsrc = 0;
        for (uint32_t i = lane; i < ec; i += kWave) {
            const uint32_t l = locs[i];
            if (l >= nd + m || (i > 0 && l <= locs[i - 1])) bad = true;
            nsrc += l < nd;
        }
        for (int off = 32; off > 0; off >>= 1) nsrc += __shfl_xor(nsrc, off);
        ok = !__any(bad);
        es = uni(nsrc);
    }
    if (ok && es > kPlanCfMaxE) ok = false;  // launch_rs_plan only picks this kernel when e fits
    if (!ok) status = 0;
    if (ok && es > 0) {
        // surviving parities in ascending slot order (reference scan normEncoderRS8.cpp:660-718);
        // the es-th survivor lies before parity offset ec, so with ec <= kPlanCfScan the lanes
        // scan 64 offsets at a time against a bitmap of the lost ones
        if (ec <= kPlanCfScan) {
            for (uint32_t i = lane; i < kPlanCfScan / 32; i += kWave) pbits[i] = 0;
            __syncthreads();
            for (uint32_t i = es + lane; i < ec; i += kWave) {
                const uint32_t off = (uint32_t)locs[i] - nd;   // < m (checked above)
                if (off < kPlanCfScan) atomicOr(&pbits[off >> 5], 1u << (off & 31u));
            }
            __syncthreads();
            uint32_t np = 0;
            const uint32_t lim = min(m, kPlanCfScan);
            for (uint32_t base = 0; np < es && base < lim; base += kWave) {
                const uint32_t off = base + lane;
                const bool surv = off < lim && !((pbits[off >> 5] >> (off & 31u)) & 1u);
                const uint64_t mask = __ballot(surv);
                const uint32_t rank = (uint32_t)__popcll(mask & ((1ull << lane) - 1ull));
                if (surv && np + rank < es) listP[np + rank] = (uint16_t)(nd + off);
                np += (uint32_t)__popcll(mask);
            }
            if (lane == 0) np_s = min(np, es);
        } else if (lane == 0) {
            uint32_t next = es, np = 0;
            for (uint32_t s = nd; s < nd + m && np < es; ++s) {
                if (next < ec && locs[next] == s) { ++next; continue; }
                listP[np++] = (uint16_t)s;
            }
            np_s = np;
        }
        for (uint32_t i = lane; i < es; i += kWave) listE[i] = locs[i];
        __syncthreads();
        if (np_s < es) { ok = false; status = 0; }
    }
    const uint32_t e = ok ? es : 0;
    // by_row (the tower decode): every block is repaired from the stage-1 encode's z rows
    // 0..P_last (its last substitute parity row), the inverse laid out by parity row
    const bool by_row = a.by_row && a.rows1 && e > 0;
    const bool by_encode = by_row || (a.rows1 && e > 0 && nd == k && listP[e - 1] == nd + e - 1);
    const uint32_t ncol = by_row ? (uint32_t)listP[e - 1] - nd + 1u : e;  // stage-2 columns
    if (lane == 0) {
        if (a.status) a.status[b] = status;
        a.rows[b] = (int32_t)e;
        a.cols2[b] = (uint16_t)ncol;
        if (a.rows1) a.rows1[b] = by_encode ? 0 : (int32_t)e;
    }
    if (e == 0) return;

    // ---- stage-1 gather matrix and slots (blocks not repaired by encode) ----
    const uint32_t cs = a.coef_stride;
    const uint16_t* gp = reinterpret_cast<const uint16_t*>(a.gen_parity);
    for (uint32_t c = lane; c < nd && !by_encode; c += kWave) {
        uint16_t* coef1 = reinterpret_cast<uint16_t*>(a.coef1) + (uint64_t)b * k * cs;
        uint16_t* islots = a.in_slots1 + (uint64_t)b * k;
        int32_t s_idx = -1;
        {
            uint32_t lo = 0, hi = e;  // first index with listE[i] >= c
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (listE[mid] < c) lo = mid + 1;
                else hi = mid;
            }
            if (lo < e && listE[lo] == c) s_idx = (int32_t)lo;
        }
        islots[c] = s_idx >= 0 ? listP[s_idx] : (uint16_t)c;
        for (uint32_t t = 0; t < cs; ++t) {
            uint16_t v = 0;
            if (t < e) {
                if (s_idx >= 0) v = (uint16_t)((uint32_t)s_idx == t);
                else v = gp[(uint64_t)(listP[t] - nd) * k + c];
            }
            coef1[(uint64_t)c * cs + t] = v;
        }
    }

    // ---- A^-1 in closed form ----
    for (uint32_t i = lane; i < e; i += kWave) {
        const uint32_t s = listE[i];
        xs[i] = s == 0 ? (uint16_t)0 : ex[(s - 1) % (uint32_t)q];
        yt[i] = ex[(k - 1 + (listP[i] - nd)) % (uint32_t)q];  // parity row p: point alpha^(k+p-1)
    }
    __syncthreads();
    const bool small = e <= kPlanCfSmall;
    if (small) {
        if (lane < e) xxs[lane] = 0, yys[lane] = 0;
        __syncthreads();
        int32_t row = 0, sx = 0, sy = 0;
        if (lane < e) {
            const uint32_t x = xs[lane], y = yt[lane];
#pragma unroll 4
            for (uint32_t t = 0; t < e; ++t) {
                const uint32_t v = lg[x ^ yt[t]];
                Lxy[lane * kLxyStride + t] = (uint16_t)v;
                row += (int32_t)v;
            }
            for (uint32_t t = lane + 1; t < e; ++t) {
                const int32_t vx = (int32_t)lg[x ^ xs[t]], vy = (int32_t)lg[y ^ yt[t]];
                sx += vx;
                sy += vy;
                atomicAdd(&xxs[t], vx);
                atomicAdd(&yys[t], vy);
            }
        }
        __syncthreads();
        if (lane < e) {
            int32_t col = 0;
            for (uint32_t t = 0; t < e; ++t) col += (int32_t)Lxy[t * kLxyStride + lane];
            // (the s' == s terms of the original sums are lg[0] = q: 0 mod q, left out here)
            int32_t acc = (int32_t)a.lwp[listE[lane]] + row - sx - xxs[lane];
            int32_t bcc = -(int32_t)a.lw[listP[lane] - nd] + col - sy - yys[lane];
            acc %= q;
            bcc %= q;
            lA[lane] = acc < 0 ? acc + q : acc;
            lB[lane] = bcc < 0 ? bcc + q : bcc;
        }
    } else {
        for (uint32_t i = lane; i < e; i += kWave) {
            const uint32_t x = xs[i], y = yt[i];
            int32_t acc = (int32_t)a.lwp[listE[i]], bcc = -(int32_t)a.lw[listP[i] - nd];
#pragma unroll 4
            for (uint32_t t = 0; t < e; ++t) {
                acc += (int32_t)lg[x ^ yt[t]] - (int32_t)lg[x ^ xs[t]];
                bcc += (int32_t)lg[y ^ xs[t]] - (int32_t)lg[y ^ yt[t]];
            }
            // the t == i terms subtract lg[0] = q (x ^ x, y ^ y), which is 0 mod q
            acc %= q;
            bcc %= q;
            lA[i] = acc < 0 ? acc + q : acc;
            lB[i] = bcc < 0 ? bcc + q : bcc;
        }
    }
    __syncthreads();
    // lg[x_s ^ y_t]: from LDS when small
    auto lxy = [&](uint32_t s_, uint32_t t_) -> int32_t {
        return small ? (int32_t)Lxy[s_ * kLxyStride + t_] : (int32_t)lg[xs[s_] ^ yt[t_]];
    };
    uint16_t* coef2 = reinterpret_cast<uint16_t*>(a.coef2) + (uint64_t)b * (a.coef2_block ? a.coef2_block : (uint64_t)cs * cs);
    if (by_row) {
        // column = parity row P_t - nd (z row), rows s < e; the lost parity rows below P_last
        // get zero columns.  pinv[col] = t (or -1) when ncol <= kPlanCfScan, else a binary search
        const bool map = ncol <= kPlanCfScan;
        if (map) {
            for (uint32_t c = lane; c < ncol; c += kWave) pinv[c] = -1;
            __syncthreads();
            for (uint32_t t = lane; t < e; t += kWave) pinv[(uint32_t)listP[t] - nd] = (int16_t)t;
            __syncthreads();
        }
        uint32_t col = lane / e, s = lane - col * e;   // (col, s) of idx, stepped without a division
        const uint32_t dcol = kWave / e, ds = kWave - dcol * e;
        for (uint32_t idx = lane; idx < ncol * e; idx += kWave) {
            uint32_t lo;
            if (map) {
                const int32_t t = pinv[col];
                lo = t < 0 ? e : (uint32_t)t;
            } else {
                lo = 0;
                uint32_t hi = e;  // first t with listP[t] - nd >= col
                while (lo < hi) {
                    const uint32_t mid = (lo + hi) >> 1;
                    if ((uint32_t)listP[mid] - nd < col) lo = mid + 1;
                    else hi = mid;
                }
                if (lo < e && (uint32_t)listP[lo] - nd != col) lo = e;
            }
            uint16_t v = 0;
            if (lo < e) {
                int32_t l = lA[s] + lB[lo] - lxy(s, lo);
                l %= q;
                if (l < 0) l += q;
                v = ex[l];
            }
            coef2[(uint64_t)col * cs + s] = v;
            col += dcol;
            s += ds;
            if (s >= e) s -= e, ++col;
        }
    } else {
        for (uint32_t idx = lane; idx < cs * cs; idx += kWave) {
            const uint32_t t = idx / cs, s = idx % cs;  // column t (input z_t), row s (output)
            uint16_t v = 0;
            if (t < e && s < e) {
                int32_t l = lA[s] + lB[t] - lxy(s, t);
                l %= q;
                if (l < 0) l += q;
                v = ex[l];
            }
            coef2[idx] = v;
        }
    }
    uint16_t* oslots = a.out_slots2 + (uint64_t)b * k;
    for (uint32_t s = lane; s < e; s += kWave) oslots[s] = listE[s];
    if (by_encode) {
        // stage 1 computes z rows 0..ncol - 1; in overwrite mode the encode must read the erased
        // source as zero (zero_base), with accumulate it reads their contents X and stage 2,
        // writing A^-1 z = d_E ^ X over them, gives exactly the reference's XOR
        if (lane == 0) atomicMax(a.rmax, ncol);
        if (!a.zero_base) return;
        uint8_t* blk = a.zero_base + (uint64_t)b * a.zero_block_stride;
        // zero_vec: the even byte count of the symbols (a tail past the last 8-byte word too)
        const uint32_t words = a.zero_vec >> 3, tail = (a.zero_vec & 7u) >> 1;
        for (uint32_t s = 0; s < e; ++s) {
            uint2* p = reinterpret_cast<uint2*>(blk + (uint64_t)listE[s] * a.zero_seg_stride);
            for (uint32_t w = lane; w < words; w += kWave) p[w] = make_uint2(0u, 0u);
            if (lane < tail) reinterpret_cast<uint16_t*>(p + words)[lane] = 0;
        }
    }
}


// ---------------------------------------------------------------------------------
// MDP plan: one wavefront per block.
// ---------------------------------------------------------------------------------
__global__ __launch_bounds__(kWave) void mdp_plan_kernel(MdpPlanArgs a)
{
    __shared__ uint8_t ex[512];
    __shared__ uint16_t lg[256];
    __shared__ uint8_t lam[512];
    // byte-wide: slots, logs and flags are all < 255 (k + m <= 255), and the smaller LDS
    // footprint keeps more of these latency-bound waves resident
    __shared__ uint8_t surv[256];
    __shared__ uint8_t eras[256];
    __shared__ uint8_t dinv_s[256], lbeta_s[256];  // per erased row: log(Dinv_r beta_r^m), log beta_r
    __shared__ uint8_t lcol_s[256], lgam_s[256];   // per survivor: log column factor, log gamma_v
    __shared__ uint8_t ers[256];            // erased-slot flags (nvecs <= 255)
    __shared__ uint8_t loc_s[256];          // the block's erasure list (ec <= m < 255)
    __shared__ uint8_t llam[512];           // log lambda_j (0xff: lambda_j = 0)

    const uint32_t lane = threadIdx.x;
    const uint32_t b = blockIdx.x;
    const uint32_t m = a.m;
    // the erasure list is fetched first so its dependent loads overlap the table staging
    const uint32_t nd = a.num_data ? uni(a.num_data[b]) : a.k;
    const uint32_t ec = uni(a.erasure_counts[b]);
    const uint16_t* locs = a.erasure_locs + (uint64_t)b * a.erasure_stride;
    const uint32_t nvecs = nd + m;
    bool ok = nd >= 1 && nd <= a.k && ec <= m && ec <= a.erasure_stride;
    for (uint32_t i = lane; i < 510; i += kWave) ex[i] = a.exp_tab[i];
    for (uint32_t i = lane; i < 256; i += kWave) lg[i] = a.log_tab[i];
    for (uint32_t i = lane; i < 256; i += kWave) ers[i] = 0;
    auto mul = [&](uint32_t x, uint32_t y) -> uint32_t { return (x && y) ? ex[lg[x] + lg[y]] : 0u; };
    // lane-parallel validation (sorted, in range) and source-erasure count (a prefix)
    uint32_t es = 0;
    if (ok) {
        bool bad = false;
        uint32_t nsrc = 0;
        for (uint32_t i = lane; i < ec; i += kWave) {
            const uint32_t l = locs[i];
            if (l >= nvecs || (i > 0 && l <= locs[i - 1])) bad = true;
            if (l < nd) ++nsrc;
            loc_s[i] = (uint8_t)l;
        }
        for (int off = 32; off > 0; off >>= 1) nsrc += __shfl_xor(nsrc, off);
        ok = !__any(bad);
        es = uni(nsrc);
    }
    __syncthreads();
    if (!ok) {
        if (lane == 0) {
            if (a.status) a.status[b] = 0;
            a.rows[b] = 0;
            a.cols[b] = 0;
        }
        return;
    }
    if (lane == 0) {
        if (a.status) a.status[b] = (int32_t)ec;
        a.rows[b] = (int32_t)es;
    }
    if (es == 0) {
        if (lane == 0) a.cols[b] = 0;
        return;
    }
    // erasure locator: lambda(x) = prod_i (1 + X_i x), X_i = alpha^(nvecs-1-loc_i), 2m coefficients
    const uint32_t deg = 2 * m;
    for (uint32_t j = lane; j < deg; j += kWave) lam[j] = (j == 0);
    __syncthreads();
    for (uint32_t i = 0; i < ec; ++i) {
        const uint32_t X = ex[nvecs - 1 - loc_s[i]];
        uint8_t nv[8];
        uint32_t n = 0;
        for (uint32_t j = lane; j < deg; j += kWave) nv[n++] = (uint8_t)(j ? (lam[j] ^ mul(X, lam[j - 1])) : lam[0]);
        __syncthreads();
        n = 0;
        for (uint32_t j = lane; j < deg; j += kWave) lam[j] = nv[n++];
        __syncthreads();
    }
    for (uint32_t j = lane; j < deg; j += kWave) llam[j] = lam[j] ? (uint8_t)lg[lam[j]] : (uint8_t)0xff;
    // surviving slots (ballot compaction over erased-slot flags), erased source rows
    for (uint32_t i = lane; i < ec; i += kWave) {
        const uint32_t l = loc_s[i];
        ers[l] = 1;
        if (i < es) eras[i] = (uint8_t)l;
    }
    __syncthreads();
    const uint32_t ns = nvecs - ec;
    for (uint32_t v0 = 0, base = 0; v0 < nvecs; v0 += kWave) {
        const uint32_t v = v0 + lane;
        const bool alive = v < nvecs && !ers[v];
        const uint64_t bal = __ballot(alive);
        if (alive) surv[base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull))] = (uint8_t)v;
        base += (uint32_t)__popcll(bal);
    }
    if (lane == 0) a.cols[b] = (uint16_t)ns;
    __syncthreads();
    // Closed form of the Forney coefficients.  The reference's repair of erased source r from
    // survivor v is C[r][v] = Dinv_r gamma_v h, h = sum_{u<m} Lambda_u(beta_r) w^(m-1-u),
    // w = gamma_v beta_r, Lambda_u the prefix sums of the locator's coefficients.  Swapping the
    // sums, sum_{j<=u<m} w^(m-1-u) = (w^(m-j) + 1) / (w + 1), so (char 2, Lambda(beta_r) = 0, the
    // lambda_m terms cancel)
    //     h = (gamma_v beta_r)^m Lambda(1 / gamma_v) / (gamma_v beta_r + 1),
    //     C[r][v] = [Dinv_r beta_r^m] [gamma_v^(m+1) Lambda(1 / gamma_v)] / (gamma_v beta_r + 1):
    // a row factor, a column factor and a Cauchy term, O(1) table lookups per entry instead of m
    // (tests/test_mdp_algebra.py checks the identity against the sum).
    for (uint32_t r = lane; r < es; r += kWave) {
        const uint32_t kk = nvecs - 1 - eras[r];
        const uint32_t lb = (255u - kk) % 255u;  // log beta
        const uint32_t l2 = (2u * lb) % 255u;
        uint32_t denom = 0, pj = 0;  // pj = lb * (j - 1) mod 255
        for (uint32_t j = 1; j < deg; j += 2) {
            const uint32_t ll = llam[j];
            if (ll != 0xffu) denom ^= ex[ll + pj];
            pj = pj + l2 >= 255u ? pj + l2 - 255u : pj + l2;
        }
        const uint32_t dinv = denom ? ex[255u - lg[denom]] : 1u;  // GINV[0] = 1 (galois.cpp:39)
        lbeta_s[r] = (uint8_t)lb;
        dinv_s[r] = (uint8_t)((lg[dinv] + (m % 255u) * lb) % 255u);  // log(Dinv_r beta_r^m)
    }
    // column factors: log(gamma_v^(m+1) Lambda(1 / gamma_v)), Lambda of degree ec
    for (uint32_t j = lane; j < ns; j += kWave) {
        const uint32_t lgam = (nvecs - 1 - surv[j]) % 255u;
        const uint32_t step = (255u - lgam) % 255u;
        uint32_t acc = 0, pi = 0;
        for (uint32_t i = 0; i <= ec; ++i) {
            const uint32_t ll = llam[i];
            if (ll != 0xffu) acc ^= ex[ll + pi];
            pi = pi + step >= 255u ? pi + step - 255u : pi + step;
        }
        // acc != 0: 1 / gamma_v is not a root (v survived)
        lcol_s[j] = (uint8_t)(((m + 1u) % 255u * lgam + (acc ? lg[acc] : 0u)) % 255u);
        lgam_s[j] = (uint8_t)lgam;
    }
    __syncthreads();
    const uint32_t cs = a.coef_stride;
    const uint32_t nv = a.k + a.m;
    uint16_t* isl = a.in_slots + (uint64_t)b * nv;
    for (uint32_t j = lane; j < ns; j += kWave) isl[j] = surv[j];
    auto entry = [&](uint32_t r, uint32_t j) -> uint32_t {
        const uint32_t w1 = ex[lgam_s[j] + lbeta_s[r]] ^ 1u;  // gamma_v beta_r + 1, nonzero (v not erased)
        int32_t l = (int32_t)dinv_s[r] + (int32_t)lcol_s[j] - (int32_t)lg[w1];
        if (l < 0) l += 255;
        return ex[l];
    };
    if (a.coef16) {
        // pass-major snippet offsets for gen_rs8_rt.hip: pass p's rows (rs8_rt_pass_rows), 8
        // entries per column, columns contiguous
        uint16_t* c16 = a.coef16 + (uint64_t)b * a.npass16 * nv * 8u;
        const uint32_t P = rs8_rt_passes(es);
        for (uint32_t p = 0; p < P; ++p) {
            uint32_t row0, row1;
            rs8_rt_pass_rows(es, p, row0, row1);
            uint16_t* cp = c16 + (uint64_t)p * nv * 8u;
            for (uint32_t idx = lane; idx < ns * 8u; idx += kWave) {
                const uint32_t r = row0 + (idx & 7u);
                cp[idx] = (uint16_t)(r < row1 ? entry(r, idx >> 3) << 7 : 0u);
            }
        }
    } else {
        uint8_t* coef = a.coef + (uint64_t)b * nv * cs;
        for (uint32_t j = lane; j < ns; j += kWave)
            for (uint32_t r = es; r < cs; ++r) coef[(uint64_t)j * cs + r] = 0;  // padding rows
        // entries [j][r], r fastest (contiguous writes); (j, r) stepped by 64 without a division
        const uint32_t dj = kWave / es, dr = kWave - dj * es;
        uint32_t j = lane / es, r = lane - (lane / es) * es;
        for (uint32_t idx = lane; idx < es * ns; idx += kWave) {
            coef[(uint64_t)j * cs + r] = (uint8_t)entry(r, j);
            j += dj;
            r += dr;
            if (r >= es) r -= es, ++j;
        }
    }
    uint16_t* osl = a.out_slots + (uint64_t)b * (a.k + a.m);
    for (uint32_t r = lane; r < es; r += kWave) osl[r] = eras[r];
}

}  // namespace

int launch_rs_plan(const RsPlanArgs& a, hipStream_t s)
{
    if (a.nblocks == 0) return NFEC_OK;
    if (a.bits == 16 && a.lwp && a.lw && std::min(a.k, a.m) <= kPlanCfMaxE)
        hipLaunchKernelGGL(rs16_plan_cf_kernel, dim3(a.nblocks), dim3(kWave), 0, s, a);
    else if (a.bits == 8) hipLaunchKernelGGL(rs_plan_kernel<uint8_t>, dim3(a.nblocks), dim3(kWave), 0, s, a);
    else hipLaunchKernelGGL(rs_plan_kernel<uint16_t>, dim3(a.nblocks), dim3(kWave), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "rs_plan launch");
    return NFEC_OK;
}

int launch_mdp_plan(const MdpPlanArgs& a, hipStream_t s)
{
    if (a.nblocks == 0) return NFEC_OK;
    hipLaunchKernelGGL(mdp_plan_kernel, dim3(a.nblocks), dim3(kWave), 0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "mdp_plan launch");
    return NFEC_OK;
}

}  // namespace nfec

// ---------------------------------------------------------------------------------
// Closed-form RS8 plan (see RsPlan2Args): one wavefront per block, m <= 64.
// ---------------------------------------------------------------------------------
namespace nfec {
namespace {

// Intra-wave LDS hand-off: every block is one wave's, so after the shared tables are staged
// no workgroup barrier is needed; this orders the wave's LDS writes before its later reads
// (and keeps the compiler from moving them across).
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

constexpr uint32_t kPlan2Waves = 4;  // blocks per workgroup, one wave each: they share the tables (8: 63.6 vs 65.4 us, noise)

__global__ __launch_bounds__(64 * kPlan2Waves) void rs_plan2_kernel(RsPlan2Args a)
{
    __shared__ uint8_t ex[512];
    __shared__ uint16_t lg[256];
    __shared__ uint16_t lwp_s[256], lw_s[256];     // the codec's log W'(x_j), log W(y_p) (k + m <= 255)
    __shared__ uint8_t xs_w[kPlan2Waves][64], yt_w[kPlan2Waves][64];   // points of E and P
    __shared__ uint16_t sP_w[kPlan2Waves][64], sE_w[kPlan2Waves][64];
    __shared__ int32_t lA_w[kPlan2Waves][64], lB_w[kPlan2Waves][64];   // per-s / per-t log factors
    __shared__ uint8_t ers_w[kPlan2Waves][256];    // erased-slot flags (k + m <= 255)
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = uni(threadIdx.x >> 6);
    uint8_t* xs = xs_w[w];
    uint8_t* yt = yt_w[w];
    uint16_t* sP = sP_w[w];
    uint16_t* sE = sE_w[w];
    int32_t* lA = lA_w[w];
    int32_t* lB = lB_w[w];
    uint8_t* ers = ers_w[w];
    const uint32_t b = blockIdx.x * kPlan2Waves + w;
    const bool live = b < a.nblocks;
    const uint32_t k = a.k, m = a.m;
    // the erasure count and list are fetched first and together (the list's first min(stride,
    // 64) entries, whatever the count: one round trip instead of two dependent ones), so they
    // overlap the table staging; a shortened block (numData < k, normEncoderRS8.cpp:675-693) has
    // its parity at slot nd + p
    const uint16_t* locs = a.erasure_locs + (uint64_t)b * a.erasure_stride;
    const uint32_t rawl = (live && lane < a.erasure_stride) ? (uint32_t)locs[lane] : 0u;
    const uint32_t ec = live ? uni(a.erasure_counts[b]) : 0u;
    const uint32_t nd = live && a.num_data ? uni(a.num_data[b]) : k;
    bool ok = ec <= m && ec <= a.erasure_stride && nd >= 1 && nd <= k;   // then ec <= 64: one entry per lane
    const uint32_t myl = (live && ok && lane < ec) ? rawl : 0u;
    for (uint32_t i = threadIdx.x; i < 510; i += 64 * kPlan2Waves) ex[i] = a.exp_tab[i];
    for (uint32_t i = threadIdx.x; i < 256; i += 64 * kPlan2Waves) lg[i] = a.log_tab[i];
    // (the closed form's per-point constants: staged with the tables instead of gathered from
    // global memory after the erasure list, another dependent round trip)
    for (uint32_t i = threadIdx.x; i < k; i += 64 * kPlan2Waves) lwp_s[i] = a.lwp[i];
    for (uint32_t i = threadIdx.x; i < m; i += 64 * kPlan2Waves) lw_s[i] = a.lw[i];
    for (uint32_t i = lane; i < 256; i += 64) ers[i] = 0;
    __syncthreads();  // the only workgroup barrier: tables staged
    if (!live) return;
    uint32_t es = 0;
    // lane-parallel validation: sorted, in range; count source erasures (sorted list => the
    // source entries are a prefix); a valid list marks its slots in ers
    if (ok) {
        const uint32_t prev = __shfl_up(myl, 1);
        const bool bad = lane < ec && (myl >= nd + m || (lane > 0 && myl <= prev));
        es = (uint32_t)__popcll(__ballot(lane < ec && myl < nd));
        ok = !__any(bad);
    }
    wave_lds_sync();
    if (ok && lane < ec) ers[myl] = 1;
    wave_lds_sync();
    // surviving parity rows: lane p tests slot nd + p
    uint64_t surv = 0;
    if (ok) {
        surv = __ballot(lane < m && !ers[nd + lane]);
        if ((uint32_t)__popcll(surv) < es) ok = false;
    }
    const uint32_t e = ok ? es : 0;
    const uint32_t cs = a.coef_stride;
    uint32_t* emask = a.emask + (uint64_t)b * 2;
    uint32_t* psel = a.psel + (uint64_t)b * 2;
    if (lane == 0) {
        if (a.status) a.status[b] = ok ? (int32_t)ec : 0;
        a.rows[b] = (int32_t)e;
        a.cols2[b] = (uint16_t)e;
    }
    // parity map: rank of each surviving row among the first e
    uint32_t rank = (uint32_t)__popcll(surv & ((1ull << lane) - 1ull));
    const bool used = e > 0 && lane < m && ((surv >> lane) & 1ull) && rank < e;
    const uint64_t pused = __ballot(used);
    const bool fused = a.fused_rows && e > 0 && e <= 16 && (pused >> a.fused_rows) == 0ull;
    if (lane < m) a.pmap[(uint64_t)b * m + lane] = used ? (uint8_t)rank : (uint8_t)0xff;
    // erased-source bitmap (k <= 64 for the specialised kernels; others ignore it), plus the
    // columns [nd, k) of a shortened block: the repair kernels skip both (read and compute
    // nothing), which is what a shortened block's absent columns need
    const uint64_t em = e > 0 ? __ballot((lane < nd && ers[lane]) || (lane >= nd && lane < k)) : 0ull;
    if (lane == 0) {
        emask[0] = (uint32_t)em;
        emask[1] = (uint32_t)(em >> 32);
        psel[0] = (uint32_t)pused;
        psel[1] = (uint32_t)(pused >> 32);
        // a block the fused repair kernel will not take (it takes 1..16 source erasures
        // repaired from parity rows below fused_rows) opens this call's gate for the unfused kernels
        if (a.gate && e > 0 && !fused) a.gate[0] = a.gate_gen;
    }
    if (e == 0) return;
    if (used) {
        sP[rank] = (uint16_t)lane;
        const uint32_t row = k + lane;  // generator row of parity p; point alpha^(row-1)
        yt[rank] = ex[(row - 1) % 255u];
    }
    if (lane < e) {
        const uint32_t s = myl;
        sE[lane] = (uint16_t)s;
        xs[lane] = s == 0 ? 0 : ex[(s - 1) % 255u];
    }
    wave_lds_sync();
    // per-s: lA[s] = lWp(x_s) + lPP(s) - lQp(s);  per-t: lB[t] = lQ(t) - lW(t) - lD(t).
    // The e x e terms are spread over the whole wave: lane (s, q) of W = e rounded up to 16 / 32 /
    // 64 lanes per group and Q = 64 / W groups sums the terms t = q, q + Q, ..., then the groups
    // are summed across lanes (the plan is bound by its LDS instruction count: with one lane per s
    // the wave issued e rounds of six table reads at e of 64 lanes).  The s2 == s and t2 == t terms
    // are lg[0] (x ^ x), subtracted back out instead of branched on
    {
        const uint32_t W = e <= 16 ? 16u : e <= 32 ? 32u : 64u, Q = 64u / W;
        const uint32_t si = lane & (W - 1u), q = lane / W;
        int32_t acc = 0, bcc = 0;
        if (si < e) {
            const uint32_t x = xs[si], y = yt[si];
            for (uint32_t t = q; t < e; t += Q) {
                acc += (int32_t)lg[x ^ yt[t]] - (int32_t)lg[x ^ xs[t]];
                bcc += (int32_t)lg[y ^ xs[t]] - (int32_t)lg[y ^ yt[t]];
            }
        }
        for (uint32_t off = W; off < 64u; off <<= 1) {
            acc += __shfl_xor(acc, (int)off);
            bcc += __shfl_xor(bcc, (int)off);
        }
        if (q == 0 && si < e) {
            acc += (int32_t)lwp_s[sE[si]] + (int32_t)lg[0];
            bcc += (int32_t)lg[0] - (int32_t)lw_s[sP[si]];
            // reduced to [0, 255) once here, so a coefficient's exponent lA + lB - log(x ^ y) lies
            // in (-255, 510) and needs one conditional add before the doubled exp table, not a modulo
            acc %= 255;
            bcc %= 255;
            lA[si] = acc < 0 ? acc + 255 : acc;
            lB[si] = bcc < 0 ? bcc + 255 : bcc;
        }
    }
    wave_lds_sync();
    uint8_t* coef = a.coef2 + (uint64_t)b * cs * cs;
    if (fused) {
        // by parity row: 16 rows of 16 u16 (cs = 32 bytes), row sP[t] holds z_t's coefficients
        // as the fused kernel's snippet byte offsets (c << 7), unused rows zero (the fused kernel
        // applies rows 0..max used row; a zero coefficient's snippet is empty)
        uint16_t* coef16 = reinterpret_cast<uint16_t*>(coef);
        // a lane's output s = lane & 15 is the same in every round: its lA and point read once
        const uint32_t s = lane & 15u;
        const int32_t las = s < e ? lA[s] : 0;
        const uint32_t xss = s < e ? xs[s] : 0u;
        for (uint32_t row = lane >> 4; row < 16u; row += 4u) {
            const uint32_t t = (uint32_t)__popcll(pused & ((1ull << row) - 1ull));  // rank of row
            uint32_t v = 0;
            if (((pused >> row) & 1ull) && s < e) {
                int32_t l = las + lB[t] - (int32_t)lg[xss ^ yt[t]];
                if (l < 0) l += 255;
                v = ex[l];
            }
            coef16[(uint64_t)row * (cs / 2) + s] = (uint16_t)(v << 7);
        }
    } else {
        for (uint32_t idx = lane; idx < e * e; idx += 64) {
            const uint32_t t = idx / e, s = idx % e;
            int32_t l = lA[s] + lB[t] - (int32_t)lg[xs[s] ^ yt[t]];
            if (l < 0) l += 255;
            coef[(uint64_t)t * cs + s] = ex[l];
        }
    }
    if (lane < e) a.out_slots2[(uint64_t)b * k + lane] = sE[lane];
}

// RS8 plan for the runtime-coefficient repair (gen_rs8_rt.hip), any (k, m) with k + m <= 255 and
// shortened blocks, in ONE pass over the block: the erased source d_E is a linear map of the
// block's numData received columns (the surviving source and, in place of each erased one, its
// substitute parity), d_E = A^-1 (P_S + G_{S,R} d_R), so the plan writes the whole e x numData
// matrix of that map and the repair is an encode-like product, numData columns in, e rows out.
// The generator's parity rows are a scaled Cauchy matrix, G[p][j] = a_p b_j / (y_p + x_j)
// (the points and scalings behind rs_plan2_kernel's closed-form A^-1), so both parts are closed
// forms:
//   erased column j = E_r (reads parity S_r):  W[s][j] = A^-1[s][r] = exp(lA[s] + lB[r] - log(x_s + y_r))
//   received column j:   W[s][j] = (A^-1 G_{S,j})[s] = exp(lA[s] + lC[j] - log(x_s + x_j)),
//   lC[j] = log b_j + sum_s' log(x_j + x_s') - sum_t log(x_j + y_t)
// (the partial-fraction solution of a Cauchy system with one more column; lwp = -log b).  Per
// block: status and rows (e) as rs_plan_kernel<uint8_t>, the column slot list, the erased slots,
// and the matrix as the kernel's snippet offsets (u16, value << 7) in a pass-major table coef1
// [b][pass < npass][j < k][8] (Rs8RtArgs::tab_pass_stride).  One wave per block, four blocks
// per workgroup sharing the field tables.
__global__ __launch_bounds__(64 * kPlan2Waves) void rs8_plan_rt_kernel(RsPlanArgs a, uint32_t npass)
{
    constexpr uint32_t kE = 128;  // e <= min(k, m) <= 127 (k + m <= 255)
    __shared__ uint8_t ex[512];
    __shared__ uint16_t lg[256];
    __shared__ uint8_t xs_w[kPlan2Waves][kE], yt_w[kPlan2Waves][kE];
    __shared__ uint16_t sP_w[kPlan2Waves][kE], sE_w[kPlan2Waves][kE];
    __shared__ int32_t lA_w[kPlan2Waves][kE], lB_w[kPlan2Waves][kE];
    __shared__ uint8_t ers_w[kPlan2Waves][256], lC_w[kPlan2Waves][256];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = uni(threadIdx.x >> 6);
    uint8_t* xs = xs_w[w];
    uint8_t* yt = yt_w[w];
    uint16_t* sP = sP_w[w];
    uint16_t* sE = sE_w[w];
    int32_t* lA = lA_w[w];
    int32_t* lB = lB_w[w];
    uint8_t* ers = ers_w[w];
    uint8_t* lC = lC_w[w];
    const uint32_t b = blockIdx.x * kPlan2Waves + w;
    const bool live = b < a.nblocks;
    const uint32_t k = a.k, m = a.m;
    const uint32_t nd = live ? (a.num_data ? uni(a.num_data[b]) : k) : 1u;
    const uint32_t ec = live ? uni(a.erasure_counts[b]) : 0u;
    const uint16_t* locs = a.erasure_locs + (uint64_t)b * a.erasure_stride;
    const uint8_t* gex = reinterpret_cast<const uint8_t*>(a.exp_tab);
    for (uint32_t i = threadIdx.x; i < 510; i += 64 * kPlan2Waves) ex[i] = gex[i];
    for (uint32_t i = threadIdx.x; i < 256; i += 64 * kPlan2Waves) lg[i] = a.log_tab[i];
    for (uint32_t i = lane; i < 256; i += 64) ers[i] = 0;
    __syncthreads();  // the only workgroup barrier: tables staged
    if (!live) return;
    // validate (sorted, in range) and count the source erasures (a prefix of the sorted list)
    bool ok = nd >= 1 && nd <= k && ec <= m && ec <= a.erasure_stride;
    uint32_t es = 0;
    if (ok) {
        bool bad = false;
        uint32_t nsrc = 0;
        for (uint32_t i = lane; i < ec; i += 64) {
            const uint32_t l = locs[i];
            if (l >= nd + m || (i > 0 && l <= locs[i - 1])) bad = true;
            nsrc += l < nd;
        }
        for (int off = 32; off > 0; off >>= 1) nsrc += __shfl_xor(nsrc, off);
        ok = !__any(bad);
        es = uni(nsrc);
    }
    wave_lds_sync();
    if (ok)
        for (uint32_t i = lane; i < ec; i += 64) ers[locs[i]] = 1;
    wave_lds_sync();
    // the first es surviving parities in ascending slot order (reference scan :660-718)
    uint32_t np = 0;
    if (ok && es > 0) {
        for (uint32_t base = 0; base < m && np < es; base += 64) {
            const uint32_t p = base + lane;
            const bool alive = p < m && !ers[nd + p];
            const uint64_t bal = __ballot(alive);
            const uint32_t r = np + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
            if (alive && r < es) {
                sP[r] = (uint16_t)p;
                yt[r] = ex[(k - 1 + p) % 255u];  // parity row p: generator row k + p, point alpha^(k+p-1)
            }
            np += (uint32_t)__popcll(bal);
        }
        if (np < es) ok = false;  // not enough parity
    }
    const uint32_t e = ok ? es : 0;
    if (lane == 0) {
        if (a.status) a.status[b] = ok ? (int32_t)ec : 0;
        a.rows[b] = (int32_t)e;
        a.cols2[b] = (uint16_t)e;
    }
    if (e == 0) return;
    for (uint32_t i = lane; i < e; i += 64) {
        const uint32_t s = locs[i];
        sE[i] = (uint16_t)s;
        xs[i] = s == 0 ? 0 : ex[(s - 1) % 255u];
    }
    wave_lds_sync();
    // ers[j] becomes the erased column's rank r + 1 (0: received), the column slot list reads
    // the substitute parity S_r for it
    for (uint32_t i = lane; i < e; i += 64) ers[sE[i]] = (uint8_t)(i + 1);
    wave_lds_sync();
    uint16_t* isl = a.in_slots1 + (uint64_t)b * k;
    for (uint32_t j = lane; j < nd; j += 64) {
        const uint32_t r = ers[j];
        isl[j] = r ? (uint16_t)(nd + sP[r - 1]) : (uint16_t)j;
    }
    // lA, lB: A^-1[s][t] = exp(lA[s] + lB[t] - log(x_s ^ y_t)) (rs_plan2_kernel's algebra)
    for (uint32_t i = lane; i < e; i += 64) {
        const uint32_t x = xs[i], y = yt[i];
        int32_t acc = (int32_t)a.lwp[sE[i]], bcc = -(int32_t)a.lw[sP[i]];
        for (uint32_t t = 0; t < e; ++t) {
            acc += (int32_t)lg[x ^ yt[t]] - (int32_t)lg[x ^ xs[t]];
            bcc += (int32_t)lg[y ^ xs[t]] - (int32_t)lg[y ^ yt[t]];
        }
        acc += (int32_t)lg[0];  // the t == i terms subtracted lg[x ^ x] = lg[0]
        bcc += (int32_t)lg[0];
        acc %= 255;
        bcc %= 255;
        lA[i] = acc < 0 ? acc + 255 : acc;
        lB[i] = bcc < 0 ? bcc + 255 : bcc;
    }
    // lC for the received columns (x_j differs from every erased and parity point)
    for (uint32_t j = lane; j < nd; j += 64) {
        if (ers[j]) continue;
        const uint32_t x = j == 0 ? 0u : ex[j - 1];  // j < 255
        int32_t acc = -(int32_t)a.lwp[j];
        for (uint32_t t = 0; t < e; ++t) acc += (int32_t)lg[x ^ xs[t]] - (int32_t)lg[x ^ yt[t]];
        acc %= 255;
        lC[j] = (uint8_t)(acc < 0 ? acc + 255 : acc);
    }
    wave_lds_sync();
    // the matrix pass-major, as the repair kernel reads it: pass p's rows [row0, row1)
    // (rs8_rt_pass_rows), per column 8 entries (16 bytes, unused ones zero), columns contiguous
    uint16_t* c1 = reinterpret_cast<uint16_t*>(a.coef1) + (uint64_t)b * npass * k * 8u;
    const uint32_t P = rs8_rt_passes(e);
    for (uint32_t p = 0; p < P; ++p) {
        uint32_t row0, row1;
        rs8_rt_pass_rows(e, p, row0, row1);
        uint16_t* cp = c1 + (uint64_t)p * k * 8u;
        for (uint32_t idx = lane; idx < nd * 8u; idx += 64) {
            const uint32_t j = idx >> 3, s = row0 + (idx & 7u);
            uint32_t v = 0;
            if (s < row1) {
                const uint32_t r = ers[j];
                int32_t l;
                if (r)
                    l = lA[s] + lB[r - 1] - (int32_t)lg[xs[s] ^ yt[r - 1]];
                else
                    l = lA[s] + (int32_t)lC[j] - (int32_t)lg[xs[s] ^ (j == 0 ? 0u : ex[j - 1])];
                if (l < 0) l += 255;
                v = (uint32_t)ex[l] << 7;
            }
            cp[idx] = (uint16_t)v;
        }
    }
    for (uint32_t i = lane; i < e; i += 64) a.out_slots2[(uint64_t)b * k + i] = sE[i];
}

}  // namespace

int launch_rs8_plan_rt(const RsPlanArgs& a, uint32_t npass, hipStream_t s)
{
    if (a.nblocks == 0) return NFEC_OK;
    if (a.bits != 8 || a.k + a.m > 255 || !a.lwp || !a.lw || npass < rs8_rt_passes(std::min(a.k, a.m)))
        return NFEC_ENOTSUP;
    hipLaunchKernelGGL(rs8_plan_rt_kernel, dim3((a.nblocks + kPlan2Waves - 1) / kPlan2Waves), dim3(64 * kPlan2Waves),
                       0, s, a, npass);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "rs8_plan_rt launch");
    return NFEC_OK;
}

int launch_rs_plan2(const RsPlan2Args& a, hipStream_t s)
{
    if (a.nblocks == 0) return NFEC_OK;
    if (a.m > 64 || a.k + a.m > 255) return NFEC_ENOTSUP;
    hipLaunchKernelGGL(rs_plan2_kernel, dim3((a.nblocks + kPlan2Waves - 1) / kPlan2Waves), dim3(64 * kPlan2Waves),
                       0, s, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return hip_fail(e, "rs_plan2 launch");
    return NFEC_OK;
}

}  // namespace nfec
