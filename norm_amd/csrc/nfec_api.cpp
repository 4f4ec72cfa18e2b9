// nfec_api.cpp -- C ABI (include/nfec.h): codec objects and batch orchestration.
//
// A codec mirrors one NormEncoder/NormDecoder Init (reference normEncoderRS8.cpp:400-462,
// :542-649; normEncoderRS16.cpp:399-461; normEncoderMDP.cpp:56-84): it owns the generator
// (built once on the host, uploaded to HBM) and the per-value kernel tables.  Batched calls
// only enqueue kernels on the caller's stream; no host<->device traffic on the hot path.
#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <functional>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <stdexcept>
#include <thread>
#include <chrono>
#include <vector>

#include "bitslice.hpp"
#include "nfec_internal.hpp"

namespace nfec {
const char* last_error_cstr();
}

using namespace nfec;

namespace {

struct DeviceGuard {
    int prev = -1;
    bool ok = true;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != dev) ok = hipSetDevice(dev) == hipSuccess;
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

template <typename T>
struct DevBuf {
    T* p = nullptr;
    size_t n = 0;
    int reserve(size_t count)
    {
        if (count <= n) return NFEC_OK;
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
        if (hipMalloc(reinterpret_cast<void**>(&p), count * sizeof(T)) != hipSuccess) {
            (void)hipGetLastError();
            return fail(NFEC_ENOMEM, "hipMalloc failed for workspace");
        }
        n = count;
        return NFEC_OK;
    }
    void release()
    {
        if (p) (void)hipFree(p);
        p = nullptr;
        n = 0;
    }
};

constexpr uint32_t kRowPad = 32;       // coefficient rows padded (kernel row chunk multiple)
// decode blocks per planning pass: bounds the workspace (stage-1 rows z, plan matrices).
// Larger passes measured faster (fewer, fuller launches: 16k -> 64k blocks took
// decode from 2.92 to 2.77 ms per 64k blocks), so a pass is as large as 8 GiB of workspace
// allows (3 % of an MI355X's 288 GB).
// budget_bytes caps it further (decode_device: half of the device memory free plus what the
// codec already holds).  NFEC_SUBBATCH overrides (A/B runs, diagnostic library).
static uint32_t sub_batch(uint64_t ws_bytes_per_block, uint64_t budget_bytes = 8ull << 30, uint32_t max_blocks = 65536)
{
    static const long env = diag_knob("NFEC_SUBBATCH", 0, 0, 1L << 20);
    if (env > 0) return (uint32_t)std::max(256L, std::min(env, 1L << 20));
    const uint64_t cap = std::min<uint64_t>(8ull << 30, budget_bytes) / std::max<uint64_t>(ws_bytes_per_block, 1);
    return (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(max_blocks, cap));
}

uint32_t round_up(uint32_t v, uint32_t a) { return (v + a - 1) / a * a; }

}  // namespace

constexpr uint32_t kHostSlots = 3;
struct HostSlot {
    uint8_t* dev = nullptr;
    uint8_t* pin = nullptr;     // pinned staging (pageable callers, segment lists)
    uint8_t* pin_dev = nullptr; // the same staging as the device addresses it (zero-copy kernels)
    uint16_t* dmeta = nullptr;  // num_data, erasure locs, counts
    uint8_t* hmeta = nullptr;   // pinned mirror of dmeta (meta_up)
    int32_t* dstat = nullptr;
    int32_t* hstat = nullptr;   // pinned status readback
    hipStream_t st = nullptr;
    hipEvent_t done = nullptr, ev_up = nullptr, ev_cd = nullptr;
    size_t dev_bytes = 0, pin_bytes = 0, meta_bytes = 0, dstat_bytes = 0, hstat_bytes = 0, hmeta_bytes = 0;
};

// host-batch pipeline resources cached per codec (run_host_batch / run_host_vectors)
struct HostStage {
    HostSlot slot[kHostSlots];
    hipStream_t cst = nullptr;  // decode compute stream
    void release()
    {
        for (auto& s : slot) {
            if (s.st) (void)hipStreamSynchronize(s.st);
            if (s.dev) (void)hipFree(s.dev);
            if (s.pin) (void)hipHostFree(s.pin);
            if (s.dmeta) (void)hipFree(s.dmeta);
            if (s.hmeta) (void)hipHostFree(s.hmeta);
            if (s.dstat) (void)hipFree(s.dstat);
            if (s.hstat) (void)hipHostFree(s.hstat);
            if (s.done) (void)hipEventDestroy(s.done);
            if (s.ev_up) (void)hipEventDestroy(s.ev_up);
            if (s.ev_cd) (void)hipEventDestroy(s.ev_cd);
            if (s.st) (void)hipStreamDestroy(s.st);
            s = HostSlot();
        }
        if (cst) {
            (void)hipStreamSynchronize(cst);
            (void)hipStreamDestroy(cst);
            cst = nullptr;
        }
    }
};

// An asynchronous host-batch call (nfec_*_host_vectors_async): the arguments are copied at
// submission, a codec-owned worker thread runs the call, the caller polls or waits.
struct nfec_request {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    int rc = NFEC_OK;
    std::string err;  // the worker thread's error message, handed to the waiting thread
    std::function<int()> run;
};

// One worker thread per codec that has seen an async call: requests on a codec complete in
// submission order (they share the codec's staging pipeline anyway); codecs run concurrently,
// so a receiver with one decoder per remote sender (normNode.h:649) overlaps its senders.
struct AsyncQueue {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<nfec_request*> q;
    std::thread th;
    bool stop = false;
    int device = 0;

    void loop()
    {
        (void)hipSetDevice(device);
        for (;;) {
            nfec_request* r = nullptr;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty()) return;  // stop requested and drained
                r = q.front();
                q.pop_front();
            }
            const int rc = r->run();
            std::lock_guard<std::mutex> lk(r->mu);
            if (rc < 0) r->err = last_error_cstr();
            r->rc = rc;
            r->done = true;
            r->cv.notify_all();
        }
    }
    void submit(nfec_request* r)
    {
        std::lock_guard<std::mutex> lk(mu);
        if (!th.joinable()) th = std::thread([this] { loop(); });
        q.push_back(r);
        cv.notify_one();
    }
    // finishes every queued request, then stops the thread
    void shutdown()
    {
        {
            std::lock_guard<std::mutex> lk(mu);
            stop = true;
            cv.notify_all();
        }
        if (th.joinable()) th.join();
    }
};

struct nfec_codec {
    int kind = 0;
    int device = 0;
    uint32_t opts = 0;  // NFEC_OPT_* (nfec_codec_create_ex)
    uint32_t k = 0, m = 0, vec = 0, sym = 1;
    // a codec over several devices (nfec_codec_create_ex): one full single-device codec per
    // listed device.  Host batches are striped over them in contiguous block ranges; device
    // batches run on the stripe of the batch's device; per-call work on stripe 0.  The outer
    // codec keeps the shape and the generator but no device state.
    std::vector<std::unique_ptr<nfec_codec>> stripes;
    uint32_t cs = 0;  // padded parity-row count
    std::vector<uint32_t> gen;  // m x k parity rows (RS) / LFSR map for a full block (MDP)
    std::vector<uint8_t> mdp_g; // MDP generator polynomial g[0..m] (the host per-segment step)

    // device-resident state
    DevBuf<uint8_t> d_coef;      // encode coefficients, column-major [k][cs] elements
    DevBuf<uint8_t> d_gen;       // m x k row-major elements (decode plan gathers)
    DevBuf<uint32_t> d_vtab;     // 256 x 8 dwords (GF(2^8) kernels)
    DevBuf<uint8_t> d_exp;       // field exp table (2q elements)
    DevBuf<uint16_t> d_log;      // field log table (q+1)
    DevBuf<uint8_t> d_mdp_step;  // MDP single LFSR step matrix, column-major [m+1][cs]
    DevBuf<uint16_t> d_lwp, d_lw;  // RS8 closed-form plan constants: log W'(x_j), log W(y_p)
    std::vector<uint16_t> h_lwp, h_lw;  // the same on the host (nfec_decode_vectors_host)
    // RS8 / MDP products with runtime coefficients (gen_rs8_rt.hip): the generator as snippet
    // offsets [k][m] (RS8), or one [k][m] table per block length nd = 1..k (MDP, shortened)
    DevBuf<uint16_t> d_rt;
    uint64_t rt_block_bytes = 0;   // MDP: bytes per numData table
    DevBuf<uint16_t> d_sel16;      // RS16 bit-sliced encode table offsets [k][m][64] (may be absent)
    DevBuf<uint16_t> d_t3off;      // RS16 shared-table encode LDS offsets [k+1][m_pad][48]
    // RS16 products by the tower-field kernel (gen_gf16_tw.hip) instead of the shared-table one:
    // snippet offsets [k][sweep][m][2] (gf16_tw_table_elems); the Toeplitz split's products likewise
    bool tw = false;
    // NFEC_OPT_HOST_ONLY: no device, no device tables; only the host per-call paths run
    bool host_only = false;
    DevBuf<uint16_t> d_twoff, d_tmvp_tw;
    // RS16 encode by the Toeplitz split (kernels_tmvp.hip): offsets of the three products, each
    // [k/2+1][m_pad(m/2)][48], then the constants' row masks (c_j [k][16], W [m][16], G0 [m][16])
    bool tmvp = false;
    int tmvp_levels = 0;           // Karatsuba levels of the split: 1 (3 products) or 2 (9, tower kernel)
    DevBuf<uint16_t> d_tmvp_off, d_tmvp_mat;
    std::mutex tmvp_mu;            // one Toeplitz encode at a time per codec: they share w_tmvp
    DevBuf<uint8_t> w_tmvp;        // prescaled pair sums + P1 rows of a sub-batch
    hipEvent_t tmvp_done = nullptr;  // the last Toeplitz encode's end, on its stream
    // two-level encode pipeline (rs16_tmvp2_encode): a second stream of the codec's own and the
    // events that fork it from the caller's stream, stagger the sub-batches' prescales and join
    hipStream_t tmvp_s2 = nullptr;
    hipEvent_t tmvp_ev[4] = {};      // fork, join, prescale done (two, alternating)
    // device-batch encodes per path that took them (NFEC_PATH_*, nfec_codec_encode_paths)
    std::atomic<uint64_t> enc_paths[NFEC_PATH_COUNT] = {};
    std::atomic<uint64_t> dec_paths[NFEC_DPATH_COUNT] = {};  // ... and decodes (NFEC_DPATH_*)

    // decode workspace (guarded by mu)
    std::mutex mu;
    DevBuf<int32_t> w_status, w_rows, w_rows1;
    DevBuf<uint32_t> w_rmax;
    DevBuf<uint16_t> w_islots, w_oslots, w_cols;
    DevBuf<uint8_t> w_coef1, w_coef2, w_z, w_work, w_pmap;
    DevBuf<uint32_t> w_emask, w_psel, w_gate;
    DevBuf<uint16_t> w_tw2;        // RS16 decode stage 2 on the tower kernel: per-block tables
    DevBuf<uint32_t> w_rowoff;     // ... and output row offsets (TwDecTablesArgs)
    uint32_t gate_gen = 0;         // per-pass generation written into w_gate (RsPlan2Args)
    // per-call staging (nfec_encode_segment / nfec_decode_vectors, guarded by mu): one device
    // buffer and one pinned mirror of the same layout, and a stream of the codec's own, so a
    // call is one gather, one H2D, the kernels, one D2H and one scatter
    DevBuf<uint8_t> s_block;
    uint8_t* s_pin = nullptr;
    size_t s_pin_bytes = 0;
    hipStream_t s_stream = nullptr;
    // host-batch pipelines (slots, pinned staging, streams): one host-batch call at a time per
    // codec.  Separate from mu, which the decode kernels' workspace takes inside such a call.
    std::mutex stage_mu;
    HostStage stage;
    AsyncQueue async;

    ~nfec_codec()
    {
        async.shutdown();  // outstanding async requests complete before the codec goes away
        // a host-only codec (device -1) holds no device state and never starts the HIP runtime
        // (hipSetDevice(-1) would also leave an error in this thread's last-error slot)
        if (host_only || device < 0) return;
        DeviceGuard g(device);
        stage.release();
        for (auto* b : {&d_coef, &d_gen, &d_exp, &w_coef1, &w_coef2, &w_z, &w_work, &s_block, &d_mdp_step, &w_tmvp})
            b->release();
        if (s_stream) {
            (void)hipStreamSynchronize(s_stream);
            (void)hipStreamDestroy(s_stream);
        }
        if (s_pin) (void)hipHostFree(s_pin);
        d_tmvp_off.release();
        d_tmvp_mat.release();
        if (tmvp_done) (void)hipEventDestroy(tmvp_done);
        if (tmvp_s2) {
            (void)hipStreamSynchronize(tmvp_s2);
            (void)hipStreamDestroy(tmvp_s2);
        }
        for (hipEvent_t ev : tmvp_ev)
            if (ev) (void)hipEventDestroy(ev);
        d_vtab.release();
        d_log.release();
        d_lwp.release();
        d_lw.release();
        d_rt.release();
        d_sel16.release();
        d_t3off.release();
        d_twoff.release();
        d_tmvp_tw.release();
        w_pmap.release();
        w_emask.release();
        w_psel.release();
        w_gate.release();
        w_status.release();
        w_rows.release();
        w_rows1.release();
        w_rmax.release();
        w_islots.release();
        w_oslots.release();
        w_cols.release();
        w_tw2.release();
        w_rowoff.release();
    }
};

namespace {

int upload(DevBuf<uint8_t>& d, const void* src, size_t bytes)
{
    int rc = d.reserve(bytes);
    if (rc) return rc;
    NFEC_HIP(hipMemcpy(d.p, src, bytes, hipMemcpyHostToDevice));
    return NFEC_OK;
}

int host_only_fail()
{
    return fail(NFEC_EDEVICE, "host-only codec (NFEC_OPT_HOST_ONLY): no GPU path");
}

int check_batch(const nfec_codec* c, const nfec_block_batch* b)
{
    if (!c || !b) return fail(NFEC_EINVAL, "null codec or batch");
    if (c->host_only) return host_only_fail();
    if (b->nblocks == 0) return NFEC_OK;
    if (!b->blocks) return fail(NFEC_EINVAL, "null blocks pointer");
    if ((reinterpret_cast<uintptr_t>(b->blocks) & 7) || (b->seg_stride & 7) || (b->block_stride & 7))
        return fail(NFEC_EINVAL, "blocks, seg_stride and block_stride must be multiples of 8 bytes");
    if (b->seg_stride < c->vec) return fail(NFEC_EINVAL, "seg_stride < vector_size");
    if (b->block_stride < (uint64_t)(c->k + c->m) * b->seg_stride && b->nblocks > 1)
        return fail(NFEC_EINVAL, "block_stride smaller than (k+m)*seg_stride");
    return NFEC_OK;
}

// NFEC_GF16_T3=0 disables the shared-table RS16 encode (A/B runs, diagnostic library)
bool use_gf16_t3()
{
    static const bool v = diag_knob("NFEC_GF16_T3", 1) != 0;
    return v;
}

// RS16 products through the tower field (gen_gf16_tw.hip, the default since round 3) or the
// shared LDS tables (gen_gf16_t3.hip, NFEC_OPT_RS16_SHARED_TABLES: both are exact, the tests run
// both); chosen per codec, so one process can hold codecs of both kinds.  NFEC_RS16_TW=0/1
// overrides (diagnostic library).
bool use_gf16_tw(const nfec_codec* c)
{
    return diag_knob("NFEC_RS16_TW", (c->opts & NFEC_OPT_RS16_SHARED_TABLES) ? 0 : 1) != 0;
}

// one RS16 product (encode, decode stage 1) on the codec's product kernel
static int launch_rs16_product(const nfec_codec* c, const Gf16T3Args& t, hipStream_t s)
{
    return c->tw ? launch_gf16_tw_encode(t, s) : launch_gf16_t3_encode(t, s);
}

// one RS16 product on the tower kernel over a whole vector of t.vec_bytes (even) bytes: its
// 8-byte pieces on the tower kernel, the 2-6 byte tail past them on the tail kernel
// (kernels_gf16tail.hip), so any NORM vector size (segmentSize + 8) stays off the exp-table kernel
static bool rs16_tw_full_covers(const Gf16T3Args& t)
{
    const uint32_t even = t.vec_bytes & ~1u, body = even & ~7u;
    if (even == 0) return false;
    Gf16T3Args b = t;
    b.vec_bytes = body;
    return (body == 0 || gf16_tw_covers(b)) && gf16_tw_tail_covers(t, even - body);
}

static int launch_rs16_tw_full(const Gf16T3Args& t, hipStream_t s)
{
    const uint32_t even = t.vec_bytes & ~1u, body = even & ~7u;
    if (body) {
        Gf16T3Args b = t;
        b.vec_bytes = body;
        const int rc = launch_gf16_tw_encode(b, s);
        if (rc) return rc;
    }
    return launch_gf16_tw_tail(t, body, even - body, s);
}

// ---- codec construction ----
// log W'(x_j) over the k source points and log W(y_p) at the parity points: the constants of
// the closed-form plans (rs_plan2_kernel for RS8, rs16_plan_cf_kernel for RS16, the host repair)
// The closed-form plans' constants: log W'(x_j) = sum_{l != j, l < k} log(x_j + x_l) over the
// source points and log W(y_p) = sum_{l < k} log(y_p + x_l) at the parity points, with x_0 = 0,
// x_l = alpha^(l-1), y_p = alpha^(k+p-1) (normEncoderRS8.cpp:432-439).  Since
// alpha^a + alpha^b = alpha^a (1 + alpha^(b-a)), with g(d) = log(1 + alpha^d):
//   log W'(x_0)  = sum_{l=1}^{k-1} (l - 1) = (k-1)(k-2)/2
//   log W'(x_j)  = (k-1)(j-1) + sum_{d=1-j, d != 0}^{k-1-j} g(d)          (j >= 1)
//   log W(y_p)   = (k+p-1) + (k-1)(k-2)/2 + sum_{d=p+1}^{k+p-1} g(d)
// so one prefix sum of g over d in [-(k-2), k+m-2] gives all of them in O(k + m) (the direct
// sums are O(k^2 + mk): seconds at RS16's largest k).  Every d stays inside (-q, q) and is never
// 0 mod q, so 1 + alpha^d is never zero.
static void plan_constants(nfec_codec* c, const Field& f)
{
    const int64_t k = c->k, m = c->m, q = f.q;
    const int64_t lo = -(k - 2), hi = k + m - 2;  // the d range (lo <= 0 <= hi for k >= 2)
    std::vector<int64_t> pre((size_t)std::max<int64_t>(0, hi - lo + 2), 0);  // pre[i] = sum of g over [lo, lo + i)
    for (int64_t d = lo, i = 0; d <= hi; ++d, ++i) {
        const int64_t g = d == 0 ? 0 : (int64_t)f.log[1u ^ f.exp[(uint32_t)(((d % q) + q) % q)]];
        pre[(size_t)i + 1] = pre[(size_t)i] + g;
    }
    auto sum = [&](int64_t a, int64_t b) -> int64_t {  // g over [a, b] (d = 0 counts 0)
        if (b < a) return 0;
        return pre[(size_t)(b - lo + 1)] - pre[(size_t)(a - lo)];
    };
    std::vector<uint16_t> lwp(c->k), lw(c->m);
    const int64_t tri = (k - 1) * (k - 2) / 2;
    for (int64_t j = 0; j < k; ++j) {
        const int64_t v = j == 0 ? tri : (k - 1) * (j - 1) + sum(1 - j, k - 1 - j);
        lwp[(size_t)j] = (uint16_t)(v % q);
    }
    for (int64_t p = 0; p < m; ++p) lw[(size_t)p] = (uint16_t)(((k + p - 1) + tri + sum(p + 1, k + p - 1)) % q);
    c->h_lwp = lwp;
    c->h_lw = lw;
}

int build_codec(nfec_codec* c)
{
    const bool wide = c->kind == NFEC_RS16;
    c->sym = wide ? 2 : 1;
    c->cs = round_up(std::max(c->m, 1u), kRowPad);
    const Field& f = wide ? gf16() : gf8();
    if (c->host_only) {
        // what the host per-call paths read: the generator (MDP: the polynomial and the full
        // block's LFSR map) and the closed-form plan constants
        if (c->kind == NFEC_MDP) {
            if (c->k + c->m > 255 || c->m == 0) return fail(NFEC_ERANGE, "MDP: numData + numParity > 255");
            mdp_generator_poly(c->m, c->mdp_g);
            std::vector<uint8_t> map((size_t)c->m * c->k);
            mdp_encode_matrix(c->mdp_g, c->m, c->k, map.data());
            c->gen.assign(map.begin(), map.end());
            return NFEC_OK;
        }
        if (rs_generator(wide ? 16 : 8, c->k, c->m, c->gen)) return fail(NFEC_ERANGE, "RS: numData/numParity exceeds code limits");
        plan_constants(c, f);  // any shape: the host repair's closed form has no size limit
        return NFEC_OK;
    }
    if (c->kind == NFEC_MDP) {
        if (c->k + c->m > 255 || c->m == 0) return fail(NFEC_ERANGE, "MDP: numData + numParity > 255");
        std::vector<uint8_t> g;
        mdp_generator_poly(c->m, g);
        c->mdp_g = g;
        // encode matrices for every block length nd = 1..k: [nd-1][col][cs]
        std::vector<uint8_t> coef((size_t)c->k * c->k * c->cs, 0);
        std::vector<uint8_t> map((size_t)c->m * c->k);
        for (uint32_t nd = 1; nd <= c->k; ++nd) {
            mdp_encode_matrix(g, c->m, nd, map.data());
            for (uint32_t col = 0; col < nd; ++col)
                for (uint32_t r = 0; r < c->m; ++r)
                    coef[((size_t)(nd - 1) * c->k + col) * c->cs + r] = map[(size_t)r * nd + col];
            if (nd == c->k) {
                c->gen.assign(map.begin(), map.end());
            }
        }
        int rc = upload(c->d_coef, coef.data(), coef.size());
        if (rc) return rc;
        {
            // the same block maps as runtime-coefficient tables, one per nd (shortened encodes)
            const uint32_t cs = rs8_rt_col_stride(c->m) / 2;
            c->rt_block_bytes = (uint64_t)c->k * cs * 2;
            // (+ padding: the kernel's scalar-cache touch reads up to 4 columns past an entry)
            std::vector<uint16_t> t((size_t)c->k * c->k * cs + 4 * cs + 64, 0);
            for (uint32_t nd = 1; nd <= c->k; ++nd)
                for (uint32_t col = 0; col < nd; ++col)
                    for (uint32_t r = 0; r < c->m; ++r)
                        t[((size_t)(nd - 1) * c->k + col) * cs + r] =
                            (uint16_t)(coef[((size_t)(nd - 1) * c->k + col) * c->cs + r] << 7);
            if ((rc = c->d_rt.reserve(t.size()))) return rc;
            NFEC_HIP(hipMemcpy(c->d_rt.p, t.data(), t.size() * 2, hipMemcpyHostToDevice));
        }
        // one in-order Encode step: inputs [d, P0..P(m-1)] -> new P (normEncoderMDP.cpp:178-211)
        std::vector<uint8_t> step((size_t)(c->m + 1) * c->cs, 0);
        for (uint32_t i = 0; i < c->m; ++i) {
            const uint8_t gi = (i + 1 < c->m) ? g[c->m - 1 - i] : g[0];
            step[(size_t)0 * c->cs + i] = gi;              // data
            step[(size_t)1 * c->cs + i] ^= gi;             // P0 enters the feedback
            if (i + 1 < c->m) step[(size_t)(i + 2) * c->cs + i] ^= 1;  // shift P(i+1) -> P(i)
        }
        rc = upload(c->d_mdp_step, step.data(), step.size());
        if (rc) return rc;
    } else {
        const int bits = wide ? 16 : 8;
        int rc = rs_generator(bits, c->k, c->m, c->gen);
        if (rc) return fail(rc, "RS: numData/numParity exceeds code limits");
        std::vector<uint8_t> coef((size_t)c->k * c->cs * c->sym, 0);
        std::vector<uint8_t> genb((size_t)c->m * c->k * c->sym);
        for (uint32_t p = 0; p < c->m; ++p)
            for (uint32_t j = 0; j < c->k; ++j) {
                const uint32_t v = c->gen[(size_t)p * c->k + j];
                if (wide) {
                    reinterpret_cast<uint16_t*>(coef.data())[(size_t)j * c->cs + p] = (uint16_t)v;
                    reinterpret_cast<uint16_t*>(genb.data())[(size_t)p * c->k + j] = (uint16_t)v;
                } else {
                    coef[(size_t)j * c->cs + p] = (uint8_t)v;
                    genb[(size_t)p * c->k + j] = (uint8_t)v;
                }
            }
        rc = upload(c->d_coef, coef.data(), coef.size());
        if (rc) return rc;
        rc = upload(c->d_gen, genb.data(), genb.size());
        if (rc) return rc;
        if (!wide) {
            const std::vector<uint16_t> t = rs8_rt_table(c->gen, c->k, c->m);
            if ((rc = c->d_rt.reserve(t.size()))) return rc;
            NFEC_HIP(hipMemcpy(c->d_rt.p, t.data(), t.size() * 2, hipMemcpyHostToDevice));
        }
        // RS16: table offsets of the bit-sliced encode, 128 bytes per coefficient.  Every wave
        // re-reads its rows' offsets per column, so the kernel only wins while the table stays
        // cache-resident: (400, 100) is 5.3 MB and 11 % faster than the exp-table kernel,
        // (4096, 256) is 134 MB and 5 % slower.  Larger codes keep the
        // exp-table kernel.
        if (wide && (uint64_t)c->k * gf16_bs_rows_padded(c->m) * 128 <= (16ull << 20)) {
            std::vector<uint16_t> sel((size_t)c->k * gf16_bs_rows_padded(c->m) * 64);
            gf16_bs_selectors(c->gen, c->k, c->m, sel.data());
            if ((rc = c->d_sel16.reserve(sel.size()))) return rc;
            NFEC_HIP(hipMemcpy(c->d_sel16.p, sel.data(), sel.size() * 2, hipMemcpyHostToDevice));
        }
        // RS16: LDS offsets of the shared-table encode (gen_gf16_t3.hip), 96 bytes per
        // coefficient (C4, k = 4096, m = 256: 104 MB)
        if (wide && use_gf16_t3() && use_gf16_tw(c)) {
            std::vector<uint16_t> off(gf16_tw_table_elems(c->k, c->m));
            gf16_tw_offsets(c->gen, c->k, c->m, off.data());
            if ((rc = c->d_twoff.reserve(off.size()))) return rc;
            NFEC_HIP(hipMemcpy(c->d_twoff.p, off.data(), off.size() * 2, hipMemcpyHostToDevice));
            c->tw = true;
        } else if (wide && use_gf16_t3()) {
            const uint32_t mp = gf16_t3_rows_padded(c->m);
            std::vector<uint16_t> off((size_t)(c->k + 1) * mp * 48);
            gf16_t3_offsets(c->gen, c->k, c->m, off.data());
            if ((rc = c->d_t3off.reserve(off.size()))) return rc;
            NFEC_HIP(hipMemcpy(c->d_t3off.p, off.data(), off.size() * 2, hipMemcpyHostToDevice));
        }
        // RS16: the Toeplitz split of the generator, three (m/2)-row products over k/2 columns
        // (one Karatsuba level) or, on the tower kernel, nine (m/4)-row products over k/4 columns
        // (two levels) instead of one m-row product over k (kernels_tmvp.hip), where its passes
        // are fewer: NFEC_OPT_RS16_TOEPLITZ_OFF never, NFEC_OPT_RS16_TOEPLITZ_ON whenever the
        // shape allows it, at the most levels allowed (tests), neither when it pays;
        // NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL caps it at one level (NFEC_RS16_TMVP=0/1/-1 overrides,
        // diagnostic library)
        // (a vector size not a multiple of 8: the split over its 8-byte pieces, the tail kernel
        // over the last 2-6 bytes with the whole generator; tower kernel only)
        if (wide && use_gf16_t3() && ((c->vec % 8) == 0 || (c->tw && c->vec >= 8))) {
            const int mode = (int)diag_knob("NFEC_RS16_TMVP",
                                            (c->opts & NFEC_OPT_RS16_TOEPLITZ_OFF)  ? 0
                                            : (c->opts & NFEC_OPT_RS16_TOEPLITZ_ON) ? 1
                                                                                    : -1,
                                            -1, 1);
            const uint32_t rpp = kGf16T3RowsPerPass;
            // cost of each form per block, in the products' units (about one column step per
            // pass, weighted on the tower kernel by the cost of a pass of the configuration a
            // launch of that many rows takes, gf16_tw_cost): the products (3^L of m >> L rows
            // over k >> L columns, plus ~20 columns' worth of fixed work per pass), the prescale
            // (~165 per column it moves: it is HBM-bound) and the postscale (per parity row ~460
            // at one level, ~700 at two: its constant multiplies).  Fitted to the split forced
            // at 0 / 1 / 2 levels on (128, 32), (256, 64), (512, 128) and C4
            // (profiles/r05/tmvp_levels/: fastest at 0, 0, 2 and 2 levels).  A third level
            // measured slower: its prescale moves 3.4 k columns per block against 2.25 k.
            const int max_levels = (!c->tw || (c->opts & NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL)) ? 1 : 2;
            uint64_t cost[3];
            int top = 0;
            for (int L = 0; L <= 2; ++L) {
                cost[L] = ~0ull;
                const uint32_t r = c->m >> L;
                if (L > max_levels || r == 0 || (L && (c->m % (1u << L)))) continue;
                // (the shared-table kernel's column map needs chunks of a power of two)
                if (L && !c->tw && ((c->m / 2) & (c->m / 2 - 1))) continue;
                top = L;
                uint64_t np = 1;
                for (int i = 0; i < L; ++i) np *= 3;
                const uint64_t cols = (c->k >> L) + 20;
                const uint64_t prod_cost = c->tw ? np * gf16_tw_cost(r) * cols : np * ((r + rpp - 1) / rpp) * cols;
                // (the shared-table kernel keeps the round-2 rule: passes alone)
                cost[L] = prod_cost + (!c->tw ? 0ull
                                       : L == 1 ? 165ull * (c->k + c->k / 2) + 460ull * c->m
                                       : L == 2 ? 165ull * (c->k + c->k / 2 + 3ull * (c->k / 4)) + 700ull * c->m
                                                : 0ull);
            }
            int levels = 0;
            if (mode == 1) levels = top;
            else if (mode != 0)
                for (int L = 1; L <= 2; ++L)
                    if (cost[L] < cost[levels]) levels = L;
            uint32_t nprod = 1;
            for (int i = 0; i < levels; ++i) nprod *= 3;
            std::vector<uint32_t> prod[9];
            std::vector<uint16_t> cm, wm, gm;
            if (levels && rs16_tmvp_plan_levels(c->k, c->m, c->gen, levels, prod, cm, wm, gm)) {
                const uint32_t cols = c->k >> levels, rows = c->m >> levels;
                const uint32_t mp = gf16_t3_rows_padded(rows);
                const size_t one = c->tw ? gf16_tw_table_elems(cols, rows) : (size_t)(cols + 1) * mp * 48;
                std::vector<uint16_t> off(nprod * one);
                for (uint32_t e = 0; e < nprod; ++e) {
                    if (c->tw) gf16_tw_offsets(prod[e], cols, rows, off.data() + e * one);
                    else gf16_t3_offsets(prod[e], cols, rows, off.data() + e * one);
                }
                std::vector<uint16_t> mat;
                mat.insert(mat.end(), cm.begin(), cm.end());
                mat.insert(mat.end(), wm.begin(), wm.end());
                mat.insert(mat.end(), gm.begin(), gm.end());
                DevBuf<uint16_t>& dst = c->tw ? c->d_tmvp_tw : c->d_tmvp_off;
                if ((rc = dst.reserve(off.size()))) return rc;
                if ((rc = c->d_tmvp_mat.reserve(mat.size()))) return rc;
                NFEC_HIP(hipMemcpy(dst.p, off.data(), off.size() * 2, hipMemcpyHostToDevice));
                NFEC_HIP(hipMemcpy(c->d_tmvp_mat.p, mat.data(), mat.size() * 2, hipMemcpyHostToDevice));
                NFEC_HIP(hipEventCreateWithFlags(&c->tmvp_done, hipEventDisableTiming));
                c->tmvp = true;
                c->tmvp_levels = levels;
            }
        }
        plan_constants(c, f);  // the host repair (nfec_decode_vectors_host) takes any shape
        if (!wide || std::min(c->k, c->m) <= kPlanCfMaxE) {
            if ((rc = c->d_lwp.reserve(c->k))) return rc;
            if ((rc = c->d_lw.reserve(c->m))) return rc;
            NFEC_HIP(hipMemcpy(c->d_lwp.p, c->h_lwp.data(), c->h_lwp.size() * 2, hipMemcpyHostToDevice));
            NFEC_HIP(hipMemcpy(c->d_lw.p, c->h_lw.data(), c->h_lw.size() * 2, hipMemcpyHostToDevice));
        }
    }
    // field tables
    if (wide) {
        std::vector<uint16_t> ex(2 * f.q), lg(f.q + 1);
        for (uint32_t i = 0; i < 2 * f.q; ++i) ex[i] = (uint16_t)f.exp[i];
        for (uint32_t i = 0; i <= f.q; ++i) lg[i] = (uint16_t)f.log[i];
        int rc = upload(c->d_exp, ex.data(), ex.size() * 2);
        if (rc) return rc;
        rc = c->d_log.reserve(lg.size());
        if (rc) return rc;
        NFEC_HIP(hipMemcpy(c->d_log.p, lg.data(), lg.size() * 2, hipMemcpyHostToDevice));
    } else {
        std::vector<uint8_t> ex(2 * f.q);
        std::vector<uint16_t> lg(f.q + 1);
        for (uint32_t i = 0; i < 2 * f.q; ++i) ex[i] = (uint8_t)f.exp[i];
        for (uint32_t i = 0; i <= f.q; ++i) lg[i] = (uint16_t)f.log[i];
        int rc = upload(c->d_exp, ex.data(), ex.size());
        if (rc) return rc;
        rc = c->d_log.reserve(lg.size());
        if (rc) return rc;
        NFEC_HIP(hipMemcpy(c->d_log.p, lg.data(), lg.size() * 2, hipMemcpyHostToDevice));
        std::vector<uint32_t> vt(256 * 8);
        for (uint32_t v = 0; v < 256; ++v) vperm_table(v, &vt[v * 8]);
        rc = c->d_vtab.reserve(vt.size());
        if (rc) return rc;
        NFEC_HIP(hipMemcpy(c->d_vtab.p, vt.data(), vt.size() * 4, hipMemcpyHostToDevice));
    }
    return NFEC_OK;
}

// NFEC_FORCE_GENERIC=1 disables the generated bit-sliced kernels (A/B runs, diagnostic library)
bool force_generic()
{
    static const bool v = diag_knob("NFEC_FORCE_GENERIC", 0) != 0;
    return v;
}

// whether the generated bit-sliced kernels cover this RS8 shape (cached per shape; codecs on
// other host threads ask concurrently, so the answer is computed into a per-call buffer under
// a lock, never into shared scratch -- the reference's unlocked fec_initialized race,
// normEncoderRS8.cpp:379-388, is not reintroduced)
bool has_bitsliced(uint32_t k, uint32_t m)
{
    static std::mutex mu;
    static std::map<uint32_t, bool> known;
    const uint32_t key = (k << 16) | m;
    std::lock_guard<std::mutex> lk(mu);
    auto it = known.find(key);
    if (it != known.end()) return it->second;
    std::vector<uint8_t> scratch(256 * 256);
    const bool v = bitsliced_encode_generator(k, m, scratch.data()) == NFEC_OK;
    known.emplace(key, v);
    return v;
}

// tuning knobs of the bit-sliced kernels (A/B runs): bit 0 XCD-contiguous workgroup
// mapping (default on: neighbouring item groups share the 128-byte lines at their boundaries,
// so one XCD's L2 fetches them once; encode 2.38 -> 2.35 ms), bit 1 nontemporal parity stores
static uint32_t bs_flags()
{
    static const uint32_t f = (uint32_t)diag_knob("NFEC_BS_FLAGS", 1, 0, 3);
    return f;
}

// NFEC_Q4=0 (diagnostic library) replaces the 4-role-wave encode kernels (gen_rs8_q4.hip) by
// the round-1 2-role assembly kernels, which only the diagnostic library builds
static bool use_q4()
{
    static const bool v = diag_knob("NFEC_Q4", 1) != 0;
    return v;
}

// NFEC_ASM=0 (diagnostic library): compiler-allocated bit-sliced kernels only
static bool use_asm()
{
    static const bool v = diag_knob("NFEC_ASM", 1) != 0;
    return v;
}

// ---- encode on a device batch ----
// RS16 encode by the Toeplitz split (kernels_tmvp.hip): per sub-batch the prescale of the chunk
// pairs, the three shared-table products in one launch, and the postscale into the parity.
// The sub-batch scratch is the codec's, so calls are ordered: each waits (on its stream) for
// the previous one's end.
// Two Karatsuba levels (tower kernel only): the level-2 prescale writes the pair sums and the
// scaled sums into the block's scratch, launches of the nine (m/4)-row products run into the
// scratch -- each reads, through a column map, the alpha input of its last alpha level (its later
// beta level selects halves) or, with no alpha in its path, the source columns themselves (c
// folded into its coefficients) -- and the level-2 postscale combines them into the m parity rows
// (kernels_tmvp.hip; gf_host.cpp, rs16_tmvp_plan_levels, whose product paths index them).
static int rs16_tmvp2_encode(nfec_codec* c, const nfec_block_batch* b, hipStream_t s)
{
    const int L = c->tmvp_levels;
    const uint32_t k = c->k, m = c->m, r = m >> L, cols = k >> L, vec = c->vec & ~7u;
    uint32_t nprod = 1;
    for (int i = 0; i < L; ++i) nprod *= 3;
    const uint32_t prow0 = k / 2 + 3 * (k / 4);                 // first product row in the scratch
    const uint64_t per_block = (uint64_t)(prow0 + nprod * r) * vec;
    std::lock_guard<std::mutex> lk(c->tmvp_mu);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        free_b = 0;
    }
    const uint64_t budget = std::min<uint64_t>(16ull << 30, ((uint64_t)free_b + c->w_tmvp.n) / 2);
    // pipeline: the batch runs as sub-batches whose products launch has about 3,072 workgroups
    // (12 per CU), alternating between the caller's stream and the codec's second one, each
    // stream with its own half of the scratch, each prescale after the previous sub-batch's.  A
    // launch's tail (its last workgroups leave CUs idle) then fills with the other stream's
    // kernels, and the HBM-bound scale kernels run beside the issue-bound products.  Measured
    // (profiles/r06/tmvp_pipe/, one box): RS16(400,100) encode 19.6-19.8 -> 19.1 ms at 16
    // sub-batches (8: 19.2, 32: 19.3, 2-4: no gain), C4 96.3 -> 91.9 ms at 16.
    // NFEC_TMVP_PIPE (knob library): 0 this rule, 1 off, N >= 2 at least N sub-batches
    static const long pipe = diag_knob("NFEC_TMVP_PIPE", 0, 0, 64);
    uint64_t want = 1;
    if (pipe == 0) {
        const uint64_t wg_x4096 = (uint64_t)nprod * (gf16_tw_passes(r, gf16_tw_rows(r)) / 4u) * vec;  // x 4096 per block
        const uint64_t target = std::max<uint64_t>(1, 3072ull * 4096ull / std::max<uint64_t>(wg_x4096, 1));
        want = (b->nblocks + target - 1) / target;
    } else if (pipe >= 2) {
        want = (uint64_t)pipe;
    }
    const bool piped = want >= 2 && b->nblocks >= 2;
    const uint32_t nbuf = piped ? 2u : 1u;
    const uint64_t cap = std::max<uint64_t>(1, budget / nbuf / per_block);
    const uint64_t nsub = std::max<uint64_t>((b->nblocks + cap - 1) / cap, piped ? want : 1u);
    const uint32_t sb = (uint32_t)std::max<uint64_t>(1, (b->nblocks + nsub - 1) / std::max<uint64_t>(nsub, 1));
    if (c->w_tmvp.reserve((size_t)nbuf * sb * per_block) != NFEC_OK) {
        (void)hipGetLastError();
        return NFEC_ENOTSUP;  // no room for the scratch: the one-product encode takes the batch
    }
    if (piped && !c->tmvp_s2) {
        if (hipStreamCreateWithFlags(&c->tmvp_s2, hipStreamNonBlocking) != hipSuccess)
            return hip_fail(hipGetLastError(), "tmvp pipeline stream");
        for (hipEvent_t& ev : c->tmvp_ev)
            NFEC_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    }
    NFEC_HIP(hipStreamWaitEvent(s, c->tmvp_done, 0));
    bool queued = false, forked = false;
    auto leave = [&](int code) {
        // the second stream's work joins the caller's before tmvp_done, so the next encode (any
        // stream) waits for both halves of the scratch
        if (forked && (hipEventRecord(c->tmvp_ev[1], c->tmvp_s2) != hipSuccess ||
                       hipStreamWaitEvent(s, c->tmvp_ev[1], 0) != hipSuccess) && code == NFEC_OK)
            code = hip_fail(hipGetLastError(), "tmvp pipeline join");
        if (queued && hipEventRecord(c->tmvp_done, s) != hipSuccess && code == NFEC_OK)
            code = hip_fail(hipGetLastError(), "tmvp event");
        return code;
    };
    const size_t one_tw = gf16_tw_table_elems(cols, r);
    int rc;
    uint32_t sub = 0;
    for (uint32_t b0 = 0; b0 < b->nblocks; b0 += sb, ++sub) {
        const uint32_t nb = std::min(sb, b->nblocks - b0);
        uint8_t* blocks = static_cast<uint8_t*>(b->blocks) + (uint64_t)b0 * b->block_stride;
        hipStream_t st = s;
        if (piped && (sub & 1u)) {
            if (!forked) {  // the second stream starts after everything before on the caller's
                if (hipEventRecord(c->tmvp_ev[0], s) != hipSuccess ||
                    hipStreamWaitEvent(c->tmvp_s2, c->tmvp_ev[0], 0) != hipSuccess)
                    return leave(hip_fail(hipGetLastError(), "tmvp pipeline fork"));
                forked = true;
            }
            st = c->tmvp_s2;
        }
        // the previous sub-batch's prescale first (the other stream); an error leaves through
        // leave(), so tmvp_done still covers what both streams already hold
        if (piped && sub > 0 && forked && hipStreamWaitEvent(st, c->tmvp_ev[2 + ((sub - 1) & 1u)], 0) != hipSuccess)
            return leave(hip_fail(hipGetLastError(), "tmvp pipeline wait"));
        Rs16TmvpArgs a;
        a.base = blocks;
        a.block_stride = b->block_stride;
        a.seg_stride = b->seg_stride;
        a.nblocks = nb;
        a.vec = vec;
        a.k = k;
        a.cw = m / 2;
        a.hw = r;
        a.sc = c->w_tmvp.p + (piped ? (uint64_t)(sub & 1u) * sb * per_block : 0u);
        a.sc_block_stride = per_block;
        a.cmat = c->d_tmvp_mat.p;
        a.wmat = c->d_tmvp_mat.p + (size_t)k * 16;
        a.gmat = c->d_tmvp_mat.p + (size_t)(k + m) * 16;
        a.num_data = b->num_data ? b->num_data + b0 : nullptr;
        std::vector<Gf16T3Args> e(nprod);
        for (uint32_t pi = 0; pi < nprod; ++pi) {
            int dg[3] = {0, 0, 0};
            for (int l = L, t = (int)pi; l >= 1; --l, t /= 3) dg[l - 1] = t % 3;
            int last_alpha = 0;
            for (int l = 1; l <= L; ++l)
                if (dg[l - 1] == 0) last_alpha = l;
            uint32_t off = 0;  // the beta levels after the last alpha select second halves
            for (int l = last_alpha + 1; l <= L; ++l)
                if (dg[l - 1] == 1) off += m >> l;
            Gf16T3Args& g = e[pi];
            g.nblocks = nb;
            g.k = cols;
            g.m = r;
            g.vec_bytes = vec;
            g.tw = c->d_tmvp_tw.p + pi * one_tw;
            g.out_base = a.sc;
            g.out_block_stride = per_block;
            g.out_seg_stride = vec;
            g.out_slot0 = prow0 + pi * r;
            if (last_alpha == 0) {  // the source columns q m + i + off, chunks of m
                g.base = blocks;
                g.block_stride = b->block_stride;
                g.seg_stride = b->seg_stride;
                g.col_div = r;
                g.col_chunk = m;
                g.col_base = off;
                g.in_slots = k + m;
                // shortened blocks: a source slot at or past the block's numData reads zeros
                g.num_data = a.num_data;
                g.nd_limit = k;
                continue;
            }
            // the alpha input of level last_alpha (block of prefix P' = the digits before it),
            // column q (m >> last_alpha) + i + off
            uint32_t pre = 0;
            for (int l = 1; l < last_alpha; ++l) pre = pre * 3 + (uint32_t)dg[l - 1];
            const uint32_t blk = (last_alpha == 1 ? 0u : k / 2) + pre * (k >> last_alpha);  // level 1: pair sums; 2: s_X
            g.base = a.sc;
            g.block_stride = per_block;
            g.seg_stride = vec;
            g.in_slots = prow0;
            if (last_alpha == L) {
                g.col_base = blk;  // plain columns
            } else {
                g.col_div = r;
                g.col_chunk = m >> last_alpha;
                g.col_base = blk + off;
            }
        }
        // a shape the kernels do not cover shows on the first sub-batch, before any parity byte
        // is written: NFEC_ENOTSUP then hands the batch to the one-product encode
        if ((rc = launch_tmvp2_prescale(a, st)))
            return leave(rc == NFEC_ENOTSUP && b0 == 0 ? rc : fail(rc, "tmvp multi-level prescale"));
        queued = true;
        if (piped && hipEventRecord(c->tmvp_ev[2 + (sub & 1u)], st) != hipSuccess)
            return leave(hip_fail(hipGetLastError(), "tmvp pipeline event"));
        for (uint32_t e0 = 0; e0 < nprod; e0 += kTwMultiMax)
            if ((rc = launch_gf16_tw_multi(e.data() + e0, std::min<uint32_t>(kTwMultiMax, nprod - e0), st)))
                return leave(rc == NFEC_ENOTSUP && b0 == 0 && e0 == 0 ? rc : fail(rc, "tmvp multi-level products"));
        if ((rc = launch_tmvp2_postscale(a, st))) return leave(fail(rc, "tmvp multi-level postscale"));
    }
    return leave(NFEC_OK);
}

static int rs16_tmvp1_encode(nfec_codec* c, const nfec_block_batch* b, hipStream_t s);

// the split over the vector's 8-byte pieces, then (vec % 8 != 0) its last 2-6 bytes on the tail
// kernel with the whole generator: the product is the same at every byte position, so the split
// and the tail write disjoint bytes of the same parity
int rs16_tmvp_encode(nfec_codec* c, const nfec_block_batch* b, hipStream_t s)
{
    const int rc = c->tmvp_levels == 2 ? rs16_tmvp2_encode(c, b, s) : rs16_tmvp1_encode(c, b, s);
    const uint32_t even = c->vec & ~1u, body = even & ~7u;
    if (rc || even == body) return rc;
    Gf16T3Args t;
    t.base = static_cast<const uint8_t*>(b->blocks);
    t.block_stride = b->block_stride;
    t.seg_stride = b->seg_stride;
    t.nblocks = b->nblocks;
    t.k = c->k;
    t.m = c->m;
    t.vec_bytes = even;
    t.tw = c->d_twoff.p;
    t.num_data = b->num_data;
    const int tr = launch_gf16_tw_tail(t, body, even - body, s);
    return tr ? fail(tr, "tmvp vector tail") : NFEC_OK;
}

static int rs16_tmvp1_encode(nfec_codec* c, const nfec_block_batch* b, hipStream_t s)
{
    const uint32_t k = c->k, m = c->m, cw = m / 2, half = k / 2, vec = c->vec & ~7u;
    // sub-batches of at most 16 GiB of scratch (C4's 4,096 blocks: one, 12.5 GB) and at most
    // half of the device memory free now (plus the scratch this codec already holds), of equal
    // size so no launch runs a small tail batch
    const uint64_t per_block = (uint64_t)(half + cw) * vec;
    std::lock_guard<std::mutex> lk(c->tmvp_mu);
    size_t free_b = 0, total_b = 0;
    if (hipMemGetInfo(&free_b, &total_b) != hipSuccess) {
        (void)hipGetLastError();
        free_b = 0;
    }
    const uint64_t budget = std::min<uint64_t>(16ull << 30, ((uint64_t)free_b + c->w_tmvp.n) / 2);
    const uint64_t cap = std::max<uint64_t>(1, budget / per_block);
    const uint64_t nsub = (b->nblocks + cap - 1) / cap;
    const uint32_t sb = (uint32_t)std::max<uint64_t>(1, (b->nblocks + nsub - 1) / std::max<uint64_t>(nsub, 1));
    // no room for the scratch: the one-product shared-table encode (no scratch) takes the batch
    if (c->w_tmvp.reserve((size_t)sb * per_block) != NFEC_OK) {
        (void)hipGetLastError();
        return NFEC_ENOTSUP;
    }
    NFEC_HIP(hipStreamWaitEvent(s, c->tmvp_done, 0));
    // once a kernel that writes the scratch is queued, every exit records tmvp_done after it, so
    // the next Toeplitz encode (any stream) waits for it even when this one hands over
    bool queued = false;
    auto leave = [&](int code) {
        if (queued && hipEventRecord(c->tmvp_done, s) != hipSuccess && code == NFEC_OK)
            code = hip_fail(hipGetLastError(), "tmvp event");
        return code;
    };
    int rc;
    const uint32_t mp = gf16_t3_rows_padded(cw);
    const size_t one = (size_t)(half + 1) * mp * 48;
    const size_t one_tw = gf16_tw_table_elems(half, cw);
    uint32_t shift = 0;
    while ((1u << shift) < cw) ++shift;
    for (uint32_t b0 = 0; b0 < b->nblocks; b0 += sb) {
        const uint32_t nb = std::min(sb, b->nblocks - b0);
        uint8_t* blocks = static_cast<uint8_t*>(b->blocks) + (uint64_t)b0 * b->block_stride;
        Rs16TmvpArgs a;
        a.base = blocks;
        a.block_stride = b->block_stride;
        a.seg_stride = b->seg_stride;
        a.nblocks = nb;
        a.vec = vec;
        a.k = k;
        a.cw = cw;
        a.s = c->w_tmvp.p;
        a.s_block_stride = (uint64_t)half * vec;
        a.x = c->w_tmvp.p + (uint64_t)sb * half * vec;
        a.x_block_stride = (uint64_t)cw * vec;
        a.cmat = c->d_tmvp_mat.p;
        a.wmat = c->d_tmvp_mat.p + (size_t)k * 16;
        a.gmat = c->d_tmvp_mat.p + (size_t)(k + m) * 16;
        a.num_data = b->num_data ? b->num_data + b0 : nullptr;
        Gf16T3Args e[3];
        for (int i = 0; i < 3; ++i) {
            e[i].nblocks = nb;
            e[i].k = half;
            e[i].m = cw;
            e[i].m_pad = mp;
            e[i].vec_bytes = vec;
            if (c->tw) e[i].tw = c->d_tmvp_tw.p + i * one_tw;
            else e[i].offs = c->d_tmvp_off.p + i * one;
            e[i].base = blocks;
            e[i].block_stride = b->block_stride;
            e[i].seg_stride = b->seg_stride;
            e[i].out_base = blocks;
            e[i].out_block_stride = b->block_stride;
            e[i].out_seg_stride = b->seg_stride;
        }
        // P0 = A (pair sums) -> parity rows [k, k + cw)
        e[0].base = a.s;
        e[0].block_stride = a.s_block_stride;
        e[0].seg_stride = vec;
        e[0].out_slot0 = k;
        // P1 over the second column of every pair -> x rows
        e[1].col_shift = shift;
        e[1].col_mask = cw - 1;
        e[1].col_div = c->tw ? cw : 0;  // (any chunk width on the tower kernel)
        e[1].col_chunk = 2 * cw;
        e[1].col_base = cw;
        e[1].in_slots = k + m;
        e[1].out_base = a.x;
        e[1].out_block_stride = a.x_block_stride;
        e[1].out_seg_stride = vec;
        e[1].out_slot0 = 0;
        // P2 over the first column of every pair -> parity rows [k + cw, k + m)
        e[2].col_shift = shift;
        e[2].col_mask = cw - 1;
        e[2].col_div = c->tw ? cw : 0;
        e[2].col_chunk = 2 * cw;
        e[2].col_base = 0;
        e[2].in_slots = k + m;
        e[2].out_slot0 = k + cw;
        if (a.num_data) {
            // shortened blocks (tower kernel only): P1 and P2 mask the source slots at or past
            // the block's numData; P0 (over the pair sums) and P2 write the parity rows after
            // it, slot numData + r
            for (int i = 0; i < 3; ++i) {
                e[i].num_data = a.num_data;
                e[i].nd_limit = k;
            }
            e[0].nd_outputs_only = 1;
            e[0].out_slot0 = 0;
            e[0].out_after_data = 1;
            e[2].out_slot0 = cw;
            e[2].out_after_data = 1;
        }
        // a shape the kernels do not cover shows on the first sub-batch, before any parity byte
        // is written: NFEC_ENOTSUP then hands the batch to the one-product encode
        if ((rc = launch_tmvp_prescale(a, s)))
            return leave(rc == NFEC_ENOTSUP && b0 == 0 ? rc : fail(rc, "tmvp prescale"));
        queued = true;
        if ((rc = c->tw ? launch_gf16_tw_multi(e, 3, s) : launch_gf16_t3_multi(e, 3, s)))
            return leave(rc == NFEC_ENOTSUP && b0 == 0 ? rc : fail(rc, "tmvp products"));
        if ((rc = launch_tmvp_postscale(a, s))) return leave(fail(rc, "tmvp postscale"));
    }
    return leave(NFEC_OK);
}

// RS8 / MDP encode on the runtime-coefficient kernel (gen_rs8_rt.hip); NFEC_ENOTSUP for layouts
// it does not take (segment tails: vec % 8 != 0, offsets past 2^31)
int launch_rt_encode(nfec_codec* c, const nfec_block_batch* b, hipStream_t s)
{
    static const bool use_rt = diag_knob("NFEC_RT", 1) != 0;  // 0: the v_perm kernel (A/B)
    if (!use_rt || !c->d_rt.p || (c->vec & 7u)) return NFEC_ENOTSUP;
    const bool mdp = c->kind == NFEC_MDP;
    Rs8RtArgs a;
    a.in_base = static_cast<const uint8_t*>(b->blocks);
    a.in_block_stride = b->block_stride;
    a.in_seg_stride = b->seg_stride;
    a.out_base = static_cast<uint8_t*>(b->blocks);
    a.out_block_stride = b->block_stride;
    a.out_seg_stride = b->seg_stride;
    a.nblocks = b->nblocks;
    a.vec_bytes = c->vec;
    a.k = c->k;
    a.m = c->m;
    a.tab = c->d_rt.p;
    a.tab_col_stride = rs8_rt_col_stride(c->m);
    a.accumulate = (b->flags & NFEC_ACCUMULATE) ? 1u : 0u;
    if (b->num_data) {
        // RS8: flat, each lane's blocks stopping at their own numData (the generator's columns
        // are the same for every numData); MDP: per block, its table depends on numData
        a.per_block = mdp ? 1 : 0;
        a.num_data = b->num_data;
        a.out_after_data = 1;
        if (mdp) {
            a.tab_block_stride = c->rt_block_bytes;
            a.tab_by_count = 1;
        }
    } else {
        a.out_slot0 = c->k;
        if (mdp) a.tab = c->d_rt.p + (uint64_t)(c->k - 1) * (c->rt_block_bytes / 2);
    }
    return launch_rs8_rt(a, s);
}

static int encode_device_impl(nfec_codec* c, const nfec_block_batch* b, hipStream_t s, int& path)
{
    const bool acc = b->flags & NFEC_ACCUMULATE;
    if (c->kind == NFEC_RS8 && !force_generic()) {
        // bit-sliced kernel specialised to this (k, m) generator, when one was generated
        bs::EncArgs e;
        e.base = static_cast<const uint8_t*>(b->blocks);
        e.out = static_cast<uint8_t*>(b->blocks);
        e.block_stride = b->block_stride;
        e.seg_stride = b->seg_stride;
        e.nblocks = b->nblocks;
        e.vec = c->vec;
        e.num_data = b->num_data;
        e.accumulate = acc;
        e.xcd_remap = bs_flags() & 1u;
        e.nt_store = (bs_flags() >> 1) & 1u;
        // hand-allocated assembly kernels first (NFEC_ASM=0 disables them for A/B runs): the
        // 4-role-wave kernels sharing each column's transpose, then the 2-role kernels
        if (use_asm() && use_q4()) {
            path = NFEC_PATH_FIXED;
            const int rc = launch_rs8_q4_encode(c->k, c->m, e, s);
            if (rc != NFEC_ENOTSUP) return rc == NFEC_OK ? NFEC_OK : fail(rc, "q4 encode launch failed");
        }
#ifdef NFEC_DIAG
        if (use_asm()) {
            const int rc = launch_rs8_asm_encode(c->k, c->m, e, s);
            if (rc != NFEC_ENOTSUP) return rc == NFEC_OK ? NFEC_OK : fail(rc, "assembly encode launch failed");
        }
#endif
        path = NFEC_PATH_FIXED;
        const int rc = launch_rs8_bitsliced_encode(c->k, c->m, e, s);
        if (rc != NFEC_ENOTSUP) return rc == NFEC_OK ? NFEC_OK : fail(rc, "bit-sliced encode launch failed");
    }
    if (c->kind == NFEC_RS8 && !force_generic()) {
        // any other shape, and shortened batches (per-block mode: the block's numData columns,
        // parity at slot numData + r): bit-sliced with runtime coefficients
        path = NFEC_PATH_RUNTIME;
        const int rc = launch_rt_encode(c, b, s);
        if (rc != NFEC_ENOTSUP) return rc;
    }
    path = NFEC_PATH_GENERIC;
    if (c->kind == NFEC_RS8) {
        Gf8MatmulArgs a;
        a.in_base = static_cast<const uint8_t*>(b->blocks);
        a.in_block_stride = b->block_stride;
        a.in_seg_stride = b->seg_stride;
        a.in_count = b->num_data;
        a.cols_const = c->k;
        a.out_base = static_cast<uint8_t*>(b->blocks);
        a.out_block_stride = b->block_stride;
        a.out_seg_stride = b->seg_stride;
        a.out_slot_mode = OUT_SLOT_AFTER_INPUT;
        a.rows_const = c->m;
        a.coef = c->d_coef.p;
        a.coef_col_stride = c->cs;
        a.vtab = c->d_vtab.p;
        a.nblocks = b->nblocks;
        a.vec_bytes = c->vec;
        a.accumulate = acc;
        return launch_gf8_matmul(a, true, s);
    }
    if (c->kind == NFEC_RS16) {
        static const bool use_bs16 = diag_knob("NFEC_GF16_BS", 1) != 0;
        // (shortened batches: on the tower kernel, whose products mask each block's source
        // slots at its numData; the prescale masks them too and the postscale writes slot
        // numData + r)
        if (c->tmvp && !acc && (!b->num_data || c->tw)) {
            path = NFEC_PATH_RS16_SPLIT;
            const int rc = rs16_tmvp_encode(c, b, s);
            if (rc != NFEC_ENOTSUP) return rc;
        }
        if (c->tw || (c->d_t3off.p && !b->num_data)) {
            // the tower kernel takes shortened batches (numData masking per 8-byte piece, parity at
            // slot numData + r) and any even vector size (tail kernel); the shared-table kernel
            // unshortened batches with vec % 8 = 0 only
            Gf16T3Args t;
            t.base = static_cast<const uint8_t*>(b->blocks);
            t.block_stride = b->block_stride;
            t.seg_stride = b->seg_stride;
            t.nblocks = b->nblocks;
            t.num_data = c->tw ? b->num_data : nullptr;
            t.k = c->k;
            t.m = c->m;
            t.m_pad = gf16_t3_rows_padded(c->m);
            t.vec_bytes = c->vec & ~1u;
            t.offs = c->d_t3off.p;
            t.tw = c->d_twoff.p;
            t.accumulate = acc;
            path = NFEC_PATH_RS16_PRODUCT;
            const int rc = !c->tw ? launch_rs16_product(c, t, s)
                           : rs16_tw_full_covers(t) ? launch_rs16_tw_full(t, s) : NFEC_ENOTSUP;
            if (rc != NFEC_ENOTSUP) return rc;
        }
        path = NFEC_PATH_GENERIC;
        if (use_bs16 && c->d_sel16.p) {
            Gf16BsEncArgs e;
            e.base = static_cast<const uint8_t*>(b->blocks);
            e.out_base = static_cast<uint8_t*>(b->blocks);
            e.block_stride = b->block_stride;
            e.seg_stride = b->seg_stride;
            e.nblocks = b->nblocks;
            e.num_data = b->num_data;
            e.k = c->k;
            e.m = c->m;
            e.vec_bytes = c->vec & ~1u;
            e.chunks = (e.vec_bytes + 63) / 64;
            e.sel = c->d_sel16.p;
            e.m_pad = gf16_bs_rows_padded(c->m);
            e.accumulate = acc;
            const int rc = launch_gf16_bs_encode(e, s);
            if (rc != NFEC_ENOTSUP) return rc;
        }
        Gf16MatmulArgs a;
        a.in_base = static_cast<const uint8_t*>(b->blocks);
        a.in_block_stride = b->block_stride;
        a.in_seg_stride = b->seg_stride;
        a.in_count = b->num_data;
        a.cols_const = c->k;
        a.out_base = static_cast<uint8_t*>(b->blocks);
        a.out_block_stride = b->block_stride;
        a.out_seg_stride = b->seg_stride;
        a.out_slot_mode = OUT_SLOT_AFTER_INPUT;
        a.rows_const = c->m;
        a.coef = reinterpret_cast<const uint16_t*>(c->d_coef.p);
        a.coef_col_stride = c->cs;
        a.exp_tab = reinterpret_cast<const uint16_t*>(c->d_exp.p);
        a.log_tab = c->d_log.p;
        a.nblocks = b->nblocks;
        a.vec_bytes = c->vec & ~1u;
        a.accumulate = acc;
        return launch_gf16_matmul(a, s);
    }
    // MDP: the in-order LFSR is a linear map of the block; the caller's parity buffers are
    // zeroed at block start by contract, so accumulate has no reference meaning.
    if (acc) return fail(NFEC_ENOTSUP, "MDP encode does not accumulate (LFSR restarts from zeroed parity)");
    if (!b->num_data && use_asm() && !force_generic()) {
        // full blocks: the LFSR's block map is a constant matrix, folded into the bit-sliced
        // assembly bodies of the RS8 encode
        bs::EncArgs e;
        e.base = static_cast<const uint8_t*>(b->blocks);
        e.out = static_cast<uint8_t*>(b->blocks);
        e.block_stride = b->block_stride;
        e.seg_stride = b->seg_stride;
        e.nblocks = b->nblocks;
        e.vec = c->vec;
        e.num_data = nullptr;
        e.accumulate = 0;
        e.xcd_remap = bs_flags() & 1u;
        e.nt_store = (bs_flags() >> 1) & 1u;
        if (use_q4()) {
            path = NFEC_PATH_FIXED;
            const int rc = launch_mdp_q4_encode(c->k, c->m, e, s);
            if (rc != NFEC_ENOTSUP) return rc == NFEC_OK ? NFEC_OK : fail(rc, "MDP q4 encode launch failed");
        }
#ifdef NFEC_DIAG
        const int rc = launch_mdp_asm_encode(c->k, c->m, e, s);
        if (rc != NFEC_ENOTSUP) return rc == NFEC_OK ? NFEC_OK : fail(rc, "MDP assembly encode launch failed");
#endif
    }
    if (!force_generic()) {
        // other shapes and shortened blocks (the block map of each block length as a table)
        path = NFEC_PATH_RUNTIME;
        const int rc = launch_rt_encode(c, b, s);
        if (rc != NFEC_ENOTSUP) return rc;
    }
    path = NFEC_PATH_GENERIC;
    Gf8MatmulArgs a;
    a.in_base = static_cast<const uint8_t*>(b->blocks);
    a.in_block_stride = b->block_stride;
    a.in_seg_stride = b->seg_stride;
    a.in_count = b->num_data;
    a.cols_const = c->k;
    a.out_base = static_cast<uint8_t*>(b->blocks);
    a.out_block_stride = b->block_stride;
    a.out_seg_stride = b->seg_stride;
    a.out_slot_mode = OUT_SLOT_AFTER_INPUT;
    a.rows_const = c->m;
    a.coef = c->d_coef.p;
    a.coef_block_stride = (uint64_t)c->k * c->cs;
    a.coef_col_stride = c->cs;
    a.coef_by_count = 1;
    a.vtab = c->d_vtab.p;
    a.nblocks = b->nblocks;
    a.vec_bytes = c->vec;
    return launch_gf8_matmul(a, false, s);
}

// counts each batch encode by the path that took it (nfec_codec_encode_paths)
int encode_device(nfec_codec* c, const nfec_block_batch* b, hipStream_t s)
{
    int path = NFEC_PATH_GENERIC;
    const int rc = encode_device_impl(c, b, s, path);
    if (rc == NFEC_OK) c->enc_paths[path].fetch_add(1, std::memory_order_relaxed);
    return rc;
}

// ---- RS16 decode on the tower kernel, every block ----
// The reference replaces each erased source row of its decoding matrix by the generator row of
// the next surviving parity (normEncoderRS16.cpp:658-716; shortened blocks :675-693) and applies
// the inverse's erased rows (:726-753).  Here, per block, with P_t the substitute parity rows
// and P_last the last of them:
//   stage 1 (flat, the encode itself): z_r = parity row r ^ sum_{c < nd} G[r][c] d_c for every
//           r <= P_last of any block (rows_lim = the batch's largest P_last + 1), with the erased
//           source read as zero (the plan zeroes it) -- so z_{P_t} = sum_s G[P_t][E_s] d_{E_s};
//           shortened blocks mask their columns at numData per 8-byte piece and read their
//           parity at slot numData + r;
//   stage 2 (per block): d_E = A^-1 z over the block's z rows 0..P_last, the inverse laid out by
//           parity row (columns of lost parity rows are zero), written over the erased source.
// With NFEC_ACCUMULATE the erased source is not zeroed: stage 1 then reads its contents X and
// z = A (d_E ^ X), so stage 2's A^-1 z = d_E ^ X written over X is the reference's XOR.  Lost
// parity (uniform loss), shortened blocks, accumulate and any even vector size (the tail kernel)
// all run here; the round-2 exp-table kernel is left for layouts past the tower kernel's 2^31
// offsets and codecs on the shared-table kernel.
static bool rs16_twdec_covers(const nfec_codec* c, const nfec_block_batch* b)
{
    static const bool on = diag_knob("NFEC_RS16_TWDEC", 1) != 0;
    if (!on || c->kind != NFEC_RS16 || !c->tw || !c->d_lwp.p || std::min(c->k, c->m) > kPlanCfMaxE) return false;
    const uint32_t zstride = round_up(c->vec, 8);
    Gf16T3Args t1;  // stage 1's layout (one block: the bounds do not depend on the count)
    t1.base = static_cast<const uint8_t*>(b->blocks);
    t1.block_stride = b->block_stride;
    t1.seg_stride = b->seg_stride;
    t1.nblocks = 1;
    t1.num_data = b->num_data;
    t1.k = c->k;
    t1.m = c->m;
    t1.vec_bytes = c->vec & ~1u;
    t1.tw = c->d_twoff.p;
    t1.accumulate = 1;
    t1.out_base = reinterpret_cast<uint8_t*>(16);  // (any non-null: the z rows' layout)
    t1.out_block_stride = (uint64_t)c->m * zstride;
    t1.out_seg_stride = zstride;
    t1.acc_base = t1.base;
    t1.acc_block_stride = b->block_stride;
    t1.acc_seg_stride = b->seg_stride;
    t1.acc_slot0 = b->num_data ? 0u : c->k;
    t1.acc_after_data = b->num_data ? 1u : 0u;
    // stage 2 writes 32-bit row offsets (erased slot * seg_stride)
    return rs16_tw_full_covers(t1) && (uint64_t)(c->k + c->m) * b->seg_stride + c->vec < (1ull << 31);
}

static int decode_rs16_tw(nfec_codec* c, const nfec_block_batch* b, const uint16_t* locs, uint32_t lstride,
                          const uint16_t* counts, int32_t* status, hipStream_t s)
{
    const bool acc = b->flags & NFEC_ACCUMULATE;
    const uint32_t zstride = round_up(c->vec, 8);
    const uint32_t M2 = std::min(c->k, c->m);              // erased source rows at most
    const uint32_t dcs = round_up(std::max(1u, M2), kRowPad);
    const uint64_t zblk = (uint64_t)c->m * zstride;        // z rows 0..m-1
    const uint64_t c2blk = (uint64_t)c->m * dcs;           // inverse by parity row: [m][dcs]
    const size_t tw2_elems = gf16_tw_table_elems(c->m, M2);  // stage-2 table: m columns, M2 rows
    const uint64_t per_block = zblk + 2ull * c2blk + 2ull * tw2_elems + 4ull * (M2 + 12) + 2ull * c->k + 64;
    uint32_t cap = std::min(b->nblocks, sub_batch(per_block, 8ull << 30, 65536u));
    const uint64_t held = c->w_z.n + c->w_coef2.n + 2ull * c->w_tw2.n;
    if ((uint64_t)cap * per_block > held) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
            cap = std::min(cap, sub_batch(per_block, ((uint64_t)free_b + held) / 2, 65536u));
        else
            (void)hipGetLastError();
    }
    const uint32_t npass = (b->nblocks + cap - 1) / std::max(cap, 1u);
    const uint32_t sb = std::max(1u, (b->nblocks + npass - 1) / std::max(npass, 1u));
    int rc;
    if ((rc = c->w_rows.reserve(sb))) return rc;
    if ((rc = c->w_rows1.reserve(sb))) return rc;
    if ((rc = c->w_cols.reserve(sb))) return rc;
    if ((rc = c->w_rmax.reserve(1))) return rc;
    if (!status && (rc = c->w_status.reserve(sb))) return rc;
    if ((rc = c->w_oslots.reserve((size_t)sb * c->k + 128))) return rc;
    if ((rc = c->w_z.reserve((size_t)sb * zblk))) return rc;
    if ((rc = c->w_coef2.reserve((size_t)sb * c2blk * 2))) return rc;
    if ((rc = c->w_tw2.reserve((size_t)sb * tw2_elems))) return rc;
    if ((rc = c->w_rowoff.reserve((size_t)sb * (M2 + 12)))) return rc;
    uint16_t phi[16];
    uint32_t lam = 0;
    gf16_tw_field(phi, &lam);
    for (uint32_t b0 = 0; b0 < b->nblocks; b0 += sb) {
        const uint32_t nb = std::min(sb, b->nblocks - b0);
        uint8_t* blocks = static_cast<uint8_t*>(b->blocks) + (uint64_t)b0 * b->block_stride;
        const uint16_t* nd = b->num_data ? b->num_data + b0 : nullptr;
        int32_t* st = status ? status + b0 : c->w_status.p;
        NFEC_HIP(hipMemsetAsync(c->w_rmax.p, 0, sizeof(uint32_t), s));
        RsPlanArgs p;
        p.bits = 16;
        p.k = c->k;
        p.m = c->m;
        p.nblocks = nb;
        p.num_data = nd;
        p.erasure_locs = locs + (uint64_t)b0 * lstride;
        p.erasure_stride = lstride;
        p.erasure_counts = counts + b0;
        p.gen_parity = c->d_gen.p;
        p.exp_tab = c->d_exp.p;
        p.log_tab = c->d_log.p;
        p.status = st;
        p.rows = c->w_rows.p;
        p.out_slots2 = c->w_oslots.p;
        p.cols2 = c->w_cols.p;
        p.coef_stride = dcs;
        p.coef2 = c->w_coef2.p;
        p.coef2_block = c2blk;
        p.lwp = c->d_lwp.p;
        p.lw = c->d_lw.p;
        p.by_row = 1;
        p.rows1 = c->w_rows1.p;
        p.rmax = c->w_rmax.p;
        p.zero_base = acc ? nullptr : blocks;
        p.zero_block_stride = b->block_stride;
        p.zero_seg_stride = b->seg_stride;
        p.zero_vec = c->vec & ~1u;
        if ((rc = launch_rs_plan(p, s))) return rc;
        // stage 1: z rows 0..rows_lim-1 of every block by the encode, XORed with its parity rows
        Gf16T3Args t;
        t.base = blocks;
        t.block_stride = b->block_stride;
        t.seg_stride = b->seg_stride;
        t.nblocks = nb;
        t.num_data = nd;
        t.k = c->k;
        t.m = c->m;
        t.vec_bytes = c->vec & ~1u;
        t.tw = c->d_twoff.p;
        t.accumulate = 1;
        t.out_base = c->w_z.p;
        t.out_block_stride = zblk;
        t.out_seg_stride = zstride;
        t.out_slot0 = 0;
        t.acc_base = blocks;
        t.acc_block_stride = b->block_stride;
        t.acc_seg_stride = b->seg_stride;
        t.acc_slot0 = nd ? 0u : c->k;
        t.acc_after_data = nd ? 1u : 0u;
        t.rows_lim = c->w_rmax.p;
        if ((rc = launch_rs16_tw_full(t, s))) return rc == NFEC_ENOTSUP ? fail(NFEC_EDEVICE, "tower decode stage 1") : rc;
        // stage 2: the per-block tables of A^-1 by parity row, then d_E = A^-1 z
        TwDecTablesArgs d;
        d.coef2 = reinterpret_cast<const uint16_t*>(c->w_coef2.p);
        d.dcs = dcs;
        d.coef2_block = c2blk;
        d.rows = c->w_rows.p;
        d.cols = c->w_cols.p;
        d.out_slots = c->w_oslots.p;
        d.slots_stride = c->k;
        d.seg_stride = b->seg_stride;
        d.nblocks = nb;
        d.M = M2;
        d.tw = c->w_tw2.p;
        d.tw_block_stride = tw2_elems;
        d.row_off = c->w_rowoff.p;
        std::copy(phi, phi + 16, d.phi);
        d.lam = lam;
        if ((rc = launch_tw_dec_tables(d, s))) return rc;
        Gf16T3Args t2;
        t2.base = c->w_z.p;
        t2.block_stride = zblk;
        t2.seg_stride = zstride;
        t2.nblocks = nb;
        t2.k = c->m;   // columns: z rows 0..P_last (blk_cols)
        t2.m = M2;     // rows: the block's e erased source (blk_rows)
        t2.vec_bytes = c->vec & ~1u;
        t2.tw = c->w_tw2.p;
        t2.tw_block_stride = tw2_elems;
        t2.blk_rows = c->w_rows.p;
        t2.blk_cols = c->w_cols.p;
        t2.row_off = c->w_rowoff.p;
        t2.row_off_stride = M2 + 12;
        t2.out_base = blocks;
        t2.out_block_stride = b->block_stride;
        t2.out_seg_stride = b->seg_stride;
        if ((rc = launch_rs16_tw_full(t2, s))) return rc == NFEC_ENOTSUP ? fail(NFEC_EDEVICE, "tower decode stage 2") : rc;
    }
    return NFEC_OK;
}

// ---- decode on a device batch ----
// caller_locked: the caller already holds c->mu (nfec_decode_vectors keeps it for the whole
// per-call decode, staging included)
static int decode_device_impl(nfec_codec* c, const nfec_block_batch* b, const uint16_t* locs, uint32_t lstride,
                              const uint16_t* counts, int32_t* status, hipStream_t s, bool caller_locked, int& path)
{
    if (!locs || !counts) return fail(NFEC_EINVAL, "null erasure arrays");
    const bool acc = b->flags & NFEC_ACCUMULATE;
    if (c->kind == NFEC_MDP && acc) return fail(NFEC_ENOTSUP, "MDP decode requires zero-filled erased segments");
    std::unique_lock<std::mutex> lk(c->mu, std::defer_lock);
    if (!caller_locked) lk.lock();
    if (rs16_twdec_covers(c, b)) {
        path = NFEC_DPATH_RS16_TOWER;
        return decode_rs16_tw(c, b, locs, lstride, counts, status, s);
    }
    const uint32_t n = c->k + c->m;
    const uint32_t zstride = round_up(c->vec, 8);
    // RS decode rows: at most min(k, m) source erasures are solved per block, so the plan's
    // matrices and the z rows are sized by that, not by m (m >> k codes, e.g. npc's auto mode)
    const uint32_t dcs = c->kind == NFEC_MDP ? c->cs : round_up(std::max(1u, std::min(c->k, c->m)), kRowPad);
    const bool big_plan = c->kind != NFEC_MDP && std::min(c->k, c->m) > 64;
    // RS8 blocks the fused / fixed-shape kernels do not take: a closed-form plan writes each
    // block's whole repair map (e x numData, rs8_plan_rt_kernel) as a pass-major snippet table
    // (8 rows per pass, 16 bytes per column) and ONE pass of the runtime-coefficient kernel
    // computes the erased source from the received columns
    // (NFEC_RT_DEC=1: the one-pass runtime-coefficient repair for those shapes too, for A/B)
    static const bool rt_first = diag_knob("NFEC_RT_DEC", 0) != 0;
    // (shortened batches too: the plan marks each block's columns past its numData like erased
    // ones, and the repair kernels read its parity at slot numData + t)
    const bool fast = !rt_first && c->kind == NFEC_RS8 && c->m <= 32 && c->k <= 64 && !force_generic() &&
                      has_bitsliced(c->k, c->m) && bs::offsets_fit(b->block_stride, b->seg_stride);
    static const bool use_rt = diag_knob("NFEC_RT", 1) != 0;
    const bool rt_dec = use_rt && !fast && c->kind == NFEC_RS8 && (c->vec % 8) == 0 && c->d_rt.p && c->d_lwp.p &&
                        !force_generic() &&
                        b->block_stride + (uint64_t)(c->k + c->m) * b->seg_stride + c->vec < (1ull << 31);
    const uint32_t E = std::min(c->k, c->m);
    // (+ RS16 on the tower kernel: stage 2's per-block snippet tables and row offsets)
    // MDP repair on the runtime-coefficient kernel (the plan's matrix as snippet offsets, one
    // pass over the survivors), else the snippet solve / generic kernel (NFEC_MDP_RT=0)
    static const bool use_mdp_rt = diag_knob("NFEC_MDP_RT", 1) != 0;
    const uint32_t mdp_np = rs8_rt_passes(std::min(c->k, c->m));  // passes of its pass-major table
    auto mdp_rt_args = [&](uint8_t* blocks, uint32_t nb) {
        Rs8RtArgs r;
        r.in_base = blocks;
        r.in_block_stride = b->block_stride;
        r.in_seg_stride = b->seg_stride;
        r.out_base = blocks;
        r.out_block_stride = b->block_stride;
        r.out_seg_stride = b->seg_stride;
        r.nblocks = nb;
        r.vec_bytes = c->vec;
        r.k = n;                          // columns: the block's survivors, up to k + m
        r.m = std::min(c->k, c->m);       // rows: its erased source
        r.per_block = 1;
        r.blk_cols = c->w_cols.p;
        r.blk_rows = c->w_rows.p;
        r.in_slots = c->w_islots.p;
        r.in_slots_stride = n;
        r.out_slots = c->w_oslots.p;
        r.out_slots_stride = n;
        r.tab = reinterpret_cast<const uint16_t*>(c->w_coef1.p);
        r.tab_block_stride = (uint64_t)mdp_np * n * 16;
        r.tab_col_stride = 16;
        r.tab_pass_stride = (uint64_t)n * 16;
        r.slot_bound = n;
        return r;
    };
    const bool mdp_rt = c->kind == NFEC_MDP && use_mdp_rt && (c->vec % 8) == 0 && !force_generic() &&
                        rs8_rt_covers(mdp_rt_args(static_cast<uint8_t*>(b->blocks), 1));
    path = fast ? NFEC_DPATH_FIXED : (rt_dec || mdp_rt) ? NFEC_DPATH_RUNTIME : NFEC_DPATH_GENERIC;
    const uint32_t rt_np = rs8_rt_passes(std::min(c->k, c->m));  // RS8 repair table passes
    const uint64_t ws_per_block = c->kind == NFEC_MDP ? (mdp_rt ? (uint64_t)mdp_np * n * 16 : (uint64_t)n * c->cs)
                                  : rt_dec            ? (uint64_t)rt_np * c->k * 16
                                                      : (uint64_t)dcs * zstride + ((uint64_t)c->k + dcs) * dcs * c->sym +
                                                 (big_plan ? rs_plan_work_bytes(dcs, c->sym) : 0) +
                                                 (c->tw ? 2ull * gf16_tw_table_elems(E, E) + 4ull * (E + 12) : 0);
    // the runtime-coefficient repair takes passes of up to 1M blocks (its launches stay well
    // below the grid limits): small codes, many blocks, no per-pass launch and plan overhead
    const uint32_t max_pass = rt_dec ? (1u << 20) : 65536u;
    // passes of equal size, so no launch runs a small tail batch
    // passes as large as 8 GiB of workspace allows; when that would grow the workspace past what
    // the codec holds, also within half of the device memory free now (plus what it holds), so
    // a smaller GPU or several codecs per device get smaller passes instead of NFEC_ENOMEM
    const uint64_t per_block = ws_per_block + 4ull * n + 64;
    uint32_t cap = std::min(b->nblocks, sub_batch(per_block, 8ull << 30, max_pass));
    const uint64_t held = c->w_z.n + c->w_coef1.n + c->w_coef2.n + c->w_work.n + 2ull * c->w_tw2.n;
    if ((uint64_t)cap * per_block > held) {
        size_t free_b = 0, total_b = 0;
        if (hipMemGetInfo(&free_b, &total_b) == hipSuccess)
            cap = std::min(cap, sub_batch(per_block, ((uint64_t)free_b + held) / 2, max_pass));
        else
            (void)hipGetLastError();
    }
    const uint32_t npass = (b->nblocks + cap - 1) / std::max(cap, 1u);
    const uint32_t sb = std::max(1u, (b->nblocks + npass - 1) / std::max(npass, 1u));
    int rc;
    if ((rc = c->w_rows.reserve(sb))) return rc;
    if ((rc = c->w_cols.reserve(sb))) return rc;
    if (!status && (rc = c->w_status.reserve(sb))) return rc;
    // + 128: the bit-sliced solves' scalar loads read up to 128 slots past a block's list
    if ((rc = c->w_islots.reserve((size_t)sb * n + 128))) return rc;
    if ((rc = c->w_oslots.reserve((size_t)sb * n + 128))) return rc;
    if (c->kind == NFEC_MDP) {
        if ((rc = c->w_coef1.reserve(mdp_rt ? (size_t)sb * mdp_np * n * 16 + 128 : (size_t)sb * n * dcs))) return rc;
    } else if (rt_dec) {
        if ((rc = c->w_coef1.reserve((size_t)sb * rt_np * c->k * 16 + 128))) return rc;
    } else {
        if ((rc = c->w_coef1.reserve((size_t)sb * c->k * dcs * c->sym))) return rc;
        if ((rc = c->w_coef2.reserve((size_t)sb * dcs * dcs * c->sym))) return rc;
        if ((rc = c->w_z.reserve((size_t)sb * dcs * zstride))) return rc;
        if (big_plan && (rc = c->w_work.reserve((size_t)sb * rs_plan_work_bytes(dcs, c->sym)))) return rc;
    }
    // RS16 stage 1 by the shared-table encode for the blocks whose substitute parities are rows
    // 0..e-1 (RsPlanArgs::rows1): overwrite semantics only, since it zeroes the erased source
    // z_t = (encode row t of the block, erased source zeroed) ^ received parity t
    auto t3_stage1 = [&](uint8_t* blocks, uint32_t nb) {
        Gf16T3Args t;
        t.base = blocks;
        t.block_stride = b->block_stride;
        t.seg_stride = b->seg_stride;
        t.nblocks = nb;
        t.k = c->k;
        t.m = c->m;
        t.m_pad = gf16_t3_rows_padded(c->m);
        t.vec_bytes = c->vec & ~1u;
        t.offs = c->d_t3off.p;
        t.tw = c->d_twoff.p;
        t.accumulate = 1;
        t.out_base = c->w_z.p;
        t.out_block_stride = (uint64_t)dcs * zstride;
        t.out_seg_stride = zstride;
        t.out_slot0 = 0;
        t.acc_base = blocks;
        t.acc_block_stride = b->block_stride;
        t.acc_seg_stride = b->seg_stride;
        t.acc_slot0 = c->k;
        t.rows_lim = c->w_rmax.p;
        return t;
    };
    // the plan marks blocks for this stage 1 only when the kernel takes the batch's layout
    // (t3_prepare's 2^31 offset bounds); otherwise every block keeps the gather stage
    bool t3dec = c->kind == NFEC_RS16 && (c->d_t3off.p || c->tw) && !b->num_data && !acc && (c->vec % 8) == 0;
    if (t3dec) {
        const Gf16T3Args t = t3_stage1(static_cast<uint8_t*>(b->blocks), sb);
        t3dec = c->tw ? gf16_tw_covers(t) : gf16_t3_covers(t);
    }
    if (t3dec) {
        if ((rc = c->w_rows1.reserve(sb))) return rc;
        if ((rc = c->w_rmax.reserve(1))) return rc;
    }
    // RS16 stage 2 (d_E = A^-1 z) on the tower kernel in per-block mode, with the batches stage
    // 1 takes by encode (overwrite, unshortened); tables of M = min(k, m) rows per block
    const uint32_t M2 = std::min(c->k, c->m);
    const size_t tw2_elems = gf16_tw_table_elems(M2, M2);
    // (the per-block row offsets are 32-bit buffer offsets of erased source slots: slot * stride)
    const bool tw2 = t3dec && c->tw && diag_knob("NFEC_RS16_TW2", 1) != 0 &&
                     (uint64_t)c->k * b->seg_stride + c->vec < (1ull << 31);
    if (tw2) {
        if ((rc = c->w_tw2.reserve((size_t)sb * tw2_elems))) return rc;
        if ((rc = c->w_rowoff.reserve((size_t)sb * (M2 + 12)))) return rc;
    }
    if (fast) {
        if ((rc = c->w_emask.reserve((size_t)sb * 2))) return rc;
        if ((rc = c->w_psel.reserve((size_t)sb * 2))) return rc;
        if ((rc = c->w_pmap.reserve((size_t)sb * c->m))) return rc;
        if ((rc = c->w_gate.reserve(1))) return rc;
    }
    for (uint32_t b0 = 0; b0 < b->nblocks; b0 += sb) {
        const uint32_t nb = std::min(sb, b->nblocks - b0);
        uint8_t* blocks = static_cast<uint8_t*>(b->blocks) + (uint64_t)b0 * b->block_stride;
        const uint16_t* nd = b->num_data ? b->num_data + b0 : nullptr;
        const uint16_t* l = locs + (uint64_t)b0 * lstride;
        const uint16_t* cnt = counts + b0;
        int32_t* st = status ? status + b0 : c->w_status.p;
        if (c->kind == NFEC_MDP) {
            MdpPlanArgs p;
            p.k = c->k;
            p.m = c->m;
            p.nblocks = nb;
            p.num_data = nd;
            p.erasure_locs = l;
            p.erasure_stride = lstride;
            p.erasure_counts = cnt;
            p.exp_tab = c->d_exp.p;
            p.log_tab = c->d_log.p;
            p.status = st;
            p.rows = c->w_rows.p;
            p.cols = c->w_cols.p;
            p.in_slots = c->w_islots.p;
            p.out_slots = c->w_oslots.p;
            p.coef_stride = dcs;
            p.coef = c->w_coef1.p;
            if (mdp_rt) {
                p.coef16 = reinterpret_cast<uint16_t*>(c->w_coef1.p);
                p.npass16 = mdp_np;
                if ((rc = launch_mdp_plan(p, s))) return rc;
                if ((rc = launch_rs8_rt(mdp_rt_args(blocks, nb), s)))
                    return fail(rc == NFEC_ENOTSUP ? NFEC_EDEVICE : rc, "MDP runtime-coefficient repair launch failed");
                continue;
            }
            if ((rc = launch_mdp_plan(p, s))) return rc;
            // blocks with <= 16 erased source vectors: the snippet solve (NFEC_MDP_BS=0: off)
            static const bool use_mdp_bs = diag_knob("NFEC_MDP_BS", 1) != 0;
            if (use_mdp_bs) {
                MdpSolveArgs ms;
                ms.base = blocks;
                ms.block_stride = b->block_stride;
                ms.seg_stride = b->seg_stride;
                ms.nblocks = nb;
                ms.vec = c->vec;
                ms.rows = c->w_rows.p;
                ms.cols = c->w_cols.p;
                ms.in_slots = c->w_islots.p;
                ms.out_slots = c->w_oslots.p;
                ms.slots_stride = n;
                ms.coef = c->w_coef1.p;
                ms.coef_block_stride = (uint64_t)n * dcs;
                ms.coef_col_stride = dcs;
                rc = launch_mdp_solve_bs(ms, s);
                if (rc != NFEC_OK && rc != NFEC_ENOTSUP) return fail(rc, "MDP solve launch failed");
            }
            Gf8MatmulArgs a;
            a.in_base = blocks;
            a.in_block_stride = b->block_stride;
            a.in_seg_stride = b->seg_stride;
            a.in_slots = c->w_islots.p;
            a.in_count = c->w_cols.p;
            a.out_base = blocks;
            a.out_block_stride = b->block_stride;
            a.out_seg_stride = b->seg_stride;
            a.out_slots = c->w_oslots.p;
            a.out_slot_mode = OUT_SLOT_LIST;
            a.row_count = c->w_rows.p;
            a.slots_stride = n;
            a.coef = c->w_coef1.p;
            a.coef_block_stride = (uint64_t)n * dcs;
            a.coef_col_stride = dcs;
            a.vtab = c->d_vtab.p;
            a.nblocks = nb;
            a.vec_bytes = c->vec;
            if ((rc = launch_gf8_matmul(a, false, s))) return rc;
            continue;
        }
        if (fast) {
            // closed-form plan -> bit-sliced re-encode (z) -> e x e inverse (generic kernel)
            RsPlan2Args p2;
            p2.k = c->k;
            p2.m = c->m;
            p2.nblocks = nb;
            p2.num_data = nd;
            p2.erasure_locs = l;
            p2.erasure_stride = lstride;
            p2.erasure_counts = cnt;
            p2.exp_tab = c->d_exp.p;
            p2.log_tab = c->d_log.p;
            p2.lwp = c->d_lwp.p;
            p2.lw = c->d_lw.p;
            p2.status = st;
            p2.rows = c->w_rows.p;
            p2.cols2 = c->w_cols.p;
            p2.out_slots2 = c->w_oslots.p;
            p2.emask = c->w_emask.p;
            p2.psel = c->w_psel.p;
            p2.pmap = c->w_pmap.p;
            p2.coef_stride = dcs;
            p2.coef2 = c->w_coef2.p;
            // fused per-block repair for the blocks it qualifies for (NFEC_FUSED=0: off); the
            // unfused stage 1 and solve below skip the blocks it marked
            static const bool use_fused = diag_knob("NFEC_FUSED", 1) != 0;
            FdecArgs f;
            f.base = blocks;
            f.block_stride = b->block_stride;
            f.seg_stride = b->seg_stride;
            f.nblocks = nb;
            f.vec = c->vec;
            f.ips = c->vec / 8;
            f.rows = c->w_rows.p;
            f.psel = c->w_psel.p;
            f.emask = c->w_emask.p;
            f.coef = c->w_coef2.p;
            f.coef_block_stride = (uint64_t)dcs * dcs;
            f.coef_col_stride = dcs;
            f.out_slots = c->w_oslots.p;
            f.slots_stride = c->k;
            f.accumulate = acc;
            f.num_data = nd;
            // 2 (default) = compact lane-major items, idle lanes out of EXEC (1.981-1.985 vs
            // 1.989-1.998 ms, r02g); 0 = item q*64 + lane; 1 = lane L holds items 4L..4L+3
            // (strided loads: 2.16 vs 2.02 ms).  NFEC_FDEC_LANEMAJOR overrides (diagnostic library).
            static const uint32_t lane_major = (uint32_t)diag_knob("NFEC_FDEC_LANEMAJOR", 2, 0, 2);
            f.lane_major = lane_major;
            const bool fused = use_fused && rs8_fused_decode_covers(c->k, c->m, f);
            // gate: the plan writes this pass's generation into w_gate when some block needs the
            // unfused kernels; when the fused kernel ran they skip their whole launch otherwise
            const uint32_t gen = ++c->gate_gen;
            if (fused) {
                p2.gate = c->w_gate.p;
                p2.gate_gen = gen;
                p2.fused_rows = std::min(16u, c->m);  // the inverse of the blocks it takes, by row
            }
            if ((rc = launch_rs_plan2(p2, s))) return rc;
            const uint32_t* gate = nullptr;
            if (fused) {
                rc = launch_rs8_fused_decode(c->k, c->m, f, s);
                if (rc != NFEC_OK) return fail(rc == NFEC_ENOTSUP ? NFEC_EDEVICE : rc, "fused decode launch failed");
                gate = c->w_gate.p;
            }
            bs::DecArgs d;
            d.base = blocks;
            d.block_stride = b->block_stride;
            d.seg_stride = b->seg_stride;
            d.nblocks = nb;
            d.vec = c->vec;
            d.emask = c->w_emask.p;
            d.psel = c->w_psel.p;
            d.pmap = c->w_pmap.p;
            d.z = c->w_z.p;
            d.z_block_stride = (uint64_t)dcs * zstride;
            d.z_stride = zstride;
            d.xcd_remap = bs_flags() & 1u;
            d.gate = gate;
            d.gate_gen = gen;
            d.num_data = nd;
            if ((rc = launch_rs8_bitsliced_reencode(c->k, c->m, d, s))) return fail(rc, "bit-sliced re-encode launch failed");
            static const bool use_solve = diag_knob("NFEC_SOLVE", 1) != 0;
            if (!use_solve) {
                Gf8MatmulArgs g2;
                g2.in_base = c->w_z.p;
                g2.in_block_stride = (uint64_t)dcs * zstride;
                g2.in_seg_stride = zstride;
                g2.in_count = c->w_cols.p;
                g2.out_base = blocks;
                g2.out_block_stride = b->block_stride;
                g2.out_seg_stride = b->seg_stride;
                g2.out_slots = c->w_oslots.p;
                g2.out_slot_mode = OUT_SLOT_LIST;
                g2.row_count = c->w_rows.p;
                g2.slots_stride = c->k;
                g2.coef = c->w_coef2.p;
                g2.coef_block_stride = (uint64_t)dcs * dcs;
                g2.coef_col_stride = dcs;
                g2.vtab = c->d_vtab.p;
                g2.nblocks = nb;
                g2.vec_bytes = c->vec;
                g2.accumulate = acc;
                if ((rc = launch_gf8_matmul(g2, false, s))) return rc;
                continue;
            }
            Gf8SolveArgs a2;
            a2.z = c->w_z.p;
            a2.z_block_stride = (uint64_t)dcs * zstride;
            a2.z_stride = zstride;
            a2.cols = c->w_cols.p;
            a2.rows = c->w_rows.p;
            a2.out_slots = c->w_oslots.p;
            a2.slots_stride = c->k;
            a2.out = blocks;
            a2.out_block_stride = b->block_stride;
            a2.out_seg_stride = b->seg_stride;
            a2.coef = c->w_coef2.p;
            a2.coef_block_stride = (uint64_t)dcs * dcs;
            a2.coef_col_stride = dcs;
            a2.vtab = c->d_vtab.p;
            a2.nblocks = nb;
            a2.vec_bytes = c->vec;
            a2.accumulate = acc;
            a2.gate = gate;
            a2.gate_gen = gen;
            // bit-sliced snippet-table solve for blocks with <= 16 erasures (NFEC_SOLVE_BS=0: off),
            // the v_perm kernel for the rest
            static const bool use_bs = diag_knob("NFEC_SOLVE_BS", 1) != 0;
            if (use_bs) {
                rc = launch_gf8_solve_bs(a2, s);
                if (rc != NFEC_OK && rc != NFEC_ENOTSUP) return fail(rc, "bit-sliced solve launch failed");
                if (rc == NFEC_OK) {
                    if (std::min(c->m, c->k) > 16) {
                        a2.min_rows = 16;
                        if ((rc = launch_gf8_solve(a2, std::min(c->m, c->k), c->m, s))) return rc;
                    }
                    continue;
                }
            }
            if ((rc = launch_gf8_solve(a2, std::min(c->m, c->k), c->m, s))) return rc;
            continue;
        }
        RsPlanArgs p;
        p.bits = c->kind == NFEC_RS16 ? 16 : 8;
        p.k = c->k;
        p.m = c->m;
        p.nblocks = nb;
        p.num_data = nd;
        p.erasure_locs = l;
        p.erasure_stride = lstride;
        p.erasure_counts = cnt;
        p.gen_parity = c->d_gen.p;
        p.exp_tab = c->d_exp.p;
        p.log_tab = c->d_log.p;
        p.status = st;
        p.rows = c->w_rows.p;
        p.in_slots1 = c->w_islots.p;
        p.out_slots2 = c->w_oslots.p;
        p.cols2 = c->w_cols.p;
        p.coef_stride = dcs;
        p.coef1 = c->w_coef1.p;
        p.coef2 = c->w_coef2.p;
        p.work = big_plan ? c->w_work.p : nullptr;
        p.work_block_bytes = rs_plan_work_bytes(dcs, c->sym);
        // RS16: the closed-form inverse when every block's e fits it (NFEC_RS16_CF=0: Gauss-Jordan)
        static const bool use_cf16 = diag_knob("NFEC_RS16_CF", 1) != 0;
        if (c->kind == NFEC_RS16 && use_cf16 && c->d_lwp.p && std::min(c->k, c->m) <= kPlanCfMaxE) {
            p.lwp = c->d_lwp.p;
            p.lw = c->d_lw.p;
        }
        if (t3dec) {
            NFEC_HIP(hipMemsetAsync(c->w_rmax.p, 0, sizeof(uint32_t), s));
            p.rows1 = c->w_rows1.p;
            p.rmax = c->w_rmax.p;
            p.zero_base = blocks;
            p.zero_block_stride = b->block_stride;
            p.zero_seg_stride = b->seg_stride;
            p.zero_vec = c->vec & ~1u;
        }
        if (rt_dec) {
            // d_E (erased source slots out_slots2) = W x the block's nd received columns (slots
            // in_slots1: the surviving source and, for an erased one, its substitute parity)
            Rs8RtArgs r;
            r.in_base = blocks;
            r.in_block_stride = b->block_stride;
            r.in_seg_stride = b->seg_stride;
            r.out_base = blocks;
            r.out_block_stride = b->block_stride;
            r.out_seg_stride = b->seg_stride;
            r.nblocks = nb;
            r.vec_bytes = c->vec;
            r.k = c->k;
            r.m = E;
            r.per_block = 1;
            r.num_data = nd;
            r.blk_rows = c->w_rows.p;
            r.in_slots = c->w_islots.p;
            r.in_slots_stride = c->k;
            r.out_slots = c->w_oslots.p;
            r.out_slots_stride = c->k;
            r.tab = reinterpret_cast<const uint16_t*>(c->w_coef1.p);
            r.tab_block_stride = (uint64_t)rt_np * c->k * 16;
            r.tab_col_stride = 16;
            r.tab_pass_stride = (uint64_t)c->k * 16;
            r.accumulate = acc;
            r.slot_bound = c->k + c->m;
            if (!rs8_rt_covers(r))
                return fail(NFEC_ENOTSUP, "runtime-coefficient repair: batch layout past its 2^31 offsets");
            p.lwp = c->d_lwp.p;
            p.lw = c->d_lw.p;
            if ((rc = launch_rs8_plan_rt(p, rt_np, s))) return rc;
            if ((rc = launch_rs8_rt(r, s)))
                return fail(rc == NFEC_ENOTSUP ? NFEC_EDEVICE : rc, "runtime-coefficient repair launch failed");
            continue;
        }
        if ((rc = launch_rs_plan(p, s))) return rc;
        if (t3dec) {
            // z_t for t below the plan's largest such e; the gather stage then overwrites the z
            // rows of the other blocks
            rc = launch_rs16_product(c, t3_stage1(blocks, nb), s);
            if (rc == NFEC_ENOTSUP) return fail(rc, "t3 decode stage 1: layout not covered");
            if (rc) return rc;
        }
        // stage 1: z_t = parity(P_t) ^ sum_{present c} G[P_t][c] d_c  -> scratch rows
        // stage 2: d_E = A^-1 z                                          -> erased slots
        if (c->kind == NFEC_RS8) {
            Gf8MatmulArgs a;
            a.in_base = blocks;
            a.in_block_stride = b->block_stride;
            a.in_seg_stride = b->seg_stride;
            a.in_slots = c->w_islots.p;
            a.in_count = nd;
            a.cols_const = c->k;
            a.out_base = c->w_z.p;
            a.out_block_stride = (uint64_t)dcs * zstride;
            a.out_seg_stride = zstride;
            a.out_slot_mode = OUT_SLOT_ROW;
            a.row_count = c->w_rows.p;
            a.slots_stride = c->k;
            a.coef = c->w_coef1.p;
            a.coef_block_stride = (uint64_t)c->k * dcs;
            a.coef_col_stride = dcs;
            a.vtab = c->d_vtab.p;
            a.nblocks = nb;
            a.vec_bytes = c->vec;
            if ((rc = launch_gf8_matmul(a, false, s))) return rc;
            Gf8MatmulArgs a2;
            a2.in_base = c->w_z.p;
            a2.in_block_stride = (uint64_t)dcs * zstride;
            a2.in_seg_stride = zstride;
            a2.in_count = c->w_cols.p;
            a2.out_base = blocks;
            a2.out_block_stride = b->block_stride;
            a2.out_seg_stride = b->seg_stride;
            a2.out_slots = c->w_oslots.p;
            a2.out_slot_mode = OUT_SLOT_LIST;
            a2.row_count = c->w_rows.p;
            a2.slots_stride = c->k;
            a2.coef = c->w_coef2.p;
            a2.coef_block_stride = (uint64_t)dcs * dcs;
            a2.coef_col_stride = dcs;
            a2.vtab = c->d_vtab.p;
            a2.nblocks = nb;
            a2.vec_bytes = c->vec;
            a2.accumulate = acc;
            if ((rc = launch_gf8_matmul(a2, false, s))) return rc;
        } else {
            const uint32_t vb = c->vec & ~1u;
            Gf16MatmulArgs a;
            a.in_base = blocks;
            a.in_block_stride = b->block_stride;
            a.in_seg_stride = b->seg_stride;
            a.in_slots = c->w_islots.p;
            a.in_count = nd;
            a.cols_const = c->k;
            a.out_base = c->w_z.p;
            a.out_block_stride = (uint64_t)dcs * zstride;
            a.out_seg_stride = zstride;
            a.out_slot_mode = OUT_SLOT_ROW;
            a.row_count = t3dec ? c->w_rows1.p : c->w_rows.p;
            a.slots_stride = c->k;
            a.coef = reinterpret_cast<const uint16_t*>(c->w_coef1.p);
            a.coef_block_stride = (uint64_t)c->k * dcs;
            a.coef_col_stride = dcs;
            a.exp_tab = reinterpret_cast<const uint16_t*>(c->d_exp.p);
            a.log_tab = c->d_log.p;
            a.nblocks = nb;
            a.vec_bytes = vb;
            if ((rc = launch_gf16_matmul(a, s))) return rc;
            if (tw2) {
                TwDecTablesArgs d;
                d.coef2 = reinterpret_cast<const uint16_t*>(c->w_coef2.p);
                d.dcs = dcs;
                d.rows = c->w_rows.p;
                d.out_slots = c->w_oslots.p;
                d.slots_stride = c->k;
                d.seg_stride = b->seg_stride;
                d.nblocks = nb;
                d.M = M2;
                d.tw = c->w_tw2.p;
                d.tw_block_stride = tw2_elems;
                d.row_off = c->w_rowoff.p;
                gf16_tw_field(d.phi, &d.lam);
                if ((rc = launch_tw_dec_tables(d, s))) return rc;
                Gf16T3Args t;
                t.base = c->w_z.p;
                t.block_stride = (uint64_t)dcs * zstride;
                t.seg_stride = zstride;
                t.nblocks = nb;
                t.k = M2;
                t.m = M2;
                t.vec_bytes = vb;
                t.tw = c->w_tw2.p;
                t.tw_block_stride = tw2_elems;
                t.blk_rows = c->w_rows.p;
                t.row_off = c->w_rowoff.p;
                t.row_off_stride = M2 + 12;
                t.out_base = blocks;
                t.out_block_stride = b->block_stride;
                t.out_seg_stride = b->seg_stride;
                rc = launch_gf16_tw_encode(t, s);
                if (rc != NFEC_ENOTSUP) {
                    if (rc) return rc;
                    continue;
                }
            }
            Gf16MatmulArgs a2 = a;
            a2.in_base = c->w_z.p;
            a2.in_block_stride = (uint64_t)dcs * zstride;
            a2.in_seg_stride = zstride;
            a2.in_slots = nullptr;
            a2.in_count = c->w_cols.p;
            a2.out_base = blocks;
            a2.out_block_stride = b->block_stride;
            a2.out_seg_stride = b->seg_stride;
            a2.out_slots = c->w_oslots.p;
            a2.out_slot_mode = OUT_SLOT_LIST;
            a2.row_count = c->w_rows.p;
            a2.coef = reinterpret_cast<const uint16_t*>(c->w_coef2.p);
            a2.coef_block_stride = (uint64_t)dcs * dcs;
            a2.accumulate = acc;
            if ((rc = launch_gf16_matmul(a2, s))) return rc;
        }
    }
    return NFEC_OK;
}

// counts each batch decode by the path that took it (nfec_codec_decode_paths)
int decode_device(nfec_codec* c, const nfec_block_batch* b, const uint16_t* locs, uint32_t lstride,
                  const uint16_t* counts, int32_t* status, hipStream_t s, bool caller_locked = false)
{
    int path = NFEC_DPATH_GENERIC;
    const int rc = decode_device_impl(c, b, locs, lstride, counts, status, s, caller_locked, path);
    if (rc == NFEC_OK) c->dec_paths[path].fetch_add(1, std::memory_order_relaxed);
    return rc;
}

}  // namespace

// =====================================================================================
// C ABI
// =====================================================================================
extern "C" {

int nfec_abi_version(void) { return NFEC_ABI_VERSION; }

const char* nfec_last_error(void) { return last_error_cstr(); }

int nfec_device_count(void)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) {
        (void)hipGetLastError();
        return 0;
    }
    int good = 0;
    for (int d = 0; d < n; ++d) {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, d) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0)
            ++good;
    }
    return good;
}

}  // extern "C"

namespace {

int create_one(int device, int kind, uint32_t num_data, uint32_t num_parity, uint32_t vector_size, uint32_t opts,
               nfec_codec** out)
{
    if (opts & NFEC_OPT_HOST_ONLY) {
        // no device is touched: Init's math and the host per-call paths only
        std::unique_ptr<nfec_codec> c(new nfec_codec);
        c->kind = kind;
        c->device = -1;
        c->opts = opts;
        c->k = num_data;
        c->m = num_parity;
        c->vec = vector_size;
        c->host_only = true;
        c->async.device = -1;
        const int rc = build_codec(c.get());
        if (rc) return rc;
        *out = c.release();
        return NFEC_OK;
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) {
        (void)hipGetLastError();
        return fail(NFEC_EDEVICE, "no such HIP device (the MI355X path needs a GPU)");
    }
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess || std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(NFEC_EDEVICE, "device is not gfx950 (MI355X)");
    DeviceGuard g(device);
    if (!g.ok) return fail(NFEC_EDEVICE, "hipSetDevice failed");
    std::unique_ptr<nfec_codec> c(new nfec_codec);
    c->kind = kind;
    c->device = device;
    c->opts = opts;
    c->k = num_data;
    c->m = num_parity;
    c->vec = vector_size;
    c->async.device = device;  // fixed before any worker thread can read it
    int rc = build_codec(c.get());
    if (rc) return rc;
    *out = c.release();
    return NFEC_OK;
}

// the codec that runs per-call work and answers shape queries
const nfec_codec* primary(const nfec_codec* c) { return c->stripes.empty() ? c : c->stripes[0].get(); }
nfec_codec* primary(nfec_codec* c) { return c->stripes.empty() ? c : c->stripes[0].get(); }

// the stripe whose device holds a device batch (a single-device codec: itself).  Only device
// allocations name a device: a batch in host-mapped or registered host memory (which the GPU
// reads over PCIe, as a single-device codec would pass it through) or in memory HIP does not
// know runs on the first stripe, so a codec's device list does not change which batches it takes.
nfec_codec* stripe_for(nfec_codec* c, const void* dev_ptr)
{
    hipPointerAttribute_t at;
    std::memset(&at, 0, sizeof(at));
    // memory HIP does not know (plain pageable malloc: the query fails or reports it
    // unregistered) is refused -- a kernel dereferencing unmapped host memory faults the GPU
    // (no XNACK); pinned / registered host and managed memory runs on stripe 0
    if (hipPointerGetAttributes(&at, dev_ptr) != hipSuccess) {
        (void)hipGetLastError();
        return nullptr;
    }
    if (at.type != hipMemoryTypeHost && at.type != hipMemoryTypeManaged && at.type != hipMemoryTypeUnified &&
        at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeArray)
        return nullptr;
    // a one-device codec runs any memory HIP maps (its own device's, a peer's, pinned host)
    if (c->stripes.empty()) return c;
    if (at.type != hipMemoryTypeDevice && at.type != hipMemoryTypeArray) return c->stripes[0].get();
    for (auto& st : c->stripes)
        if (st->device == at.device) return st.get();
    return nullptr;
}

}  // namespace

extern "C" {

int nfec_codec_create(int device, int kind, uint32_t num_data, uint32_t num_parity, uint32_t vector_size,
                      nfec_codec** out)
{
    nfec_codec_config cfg{};
    cfg.kind = kind;
    cfg.num_data = num_data;
    cfg.num_parity = num_parity;
    cfg.vector_size = vector_size;
    const int32_t dev = device;
    cfg.devices = &dev;
    cfg.num_devices = 1;
    return nfec_codec_create_ex(&cfg, out);
}

int nfec_codec_create_ex(const nfec_codec_config* cfg, nfec_codec** out)
{
    if (!out || !cfg) return fail(NFEC_EINVAL, "null argument");
    *out = nullptr;
    const int kind = cfg->kind;
    if (kind != NFEC_RS8 && kind != NFEC_RS16 && kind != NFEC_MDP) return fail(NFEC_EINVAL, "unknown codec kind");
    if (cfg->num_data == 0 || cfg->num_parity == 0) return fail(NFEC_EINVAL, "numData and numParity must be > 0");
    if (cfg->vector_size == 0 || cfg->vector_size > 65535) return fail(NFEC_EINVAL, "vectorSize must be in [1, 65535]");
    if (cfg->flags & ~(uint32_t)(NFEC_OPT_RS16_SHARED_TABLES | NFEC_OPT_RS16_TOEPLITZ_OFF | NFEC_OPT_RS16_TOEPLITZ_ON |
                                 NFEC_OPT_HOST_ONLY | NFEC_OPT_RS16_TOEPLITZ_ONE_LEVEL))
        return fail(NFEC_EINVAL, "unknown option flag");
    if ((cfg->flags & NFEC_OPT_HOST_ONLY) && cfg->num_devices > 1)
        return fail(NFEC_EINVAL, "a host-only codec takes no device list");
    if ((cfg->flags & NFEC_OPT_RS16_TOEPLITZ_OFF) && (cfg->flags & NFEC_OPT_RS16_TOEPLITZ_ON))
        return fail(NFEC_EINVAL, "Toeplitz split both on and off");
    const uint32_t nd = cfg->num_devices ? cfg->num_devices : 1;
    if (nd > 64) return fail(NFEC_EINVAL, "more than 64 devices");
    if (cfg->num_devices > 0 && !cfg->devices) return fail(NFEC_EINVAL, "null device list");
    auto dev_at = [&](uint32_t i) { return cfg->devices ? (int)cfg->devices[i] : 0; };
    if (nd == 1) return create_one(dev_at(0), kind, cfg->num_data, cfg->num_parity, cfg->vector_size, cfg->flags, out);
    std::unique_ptr<nfec_codec> c(new nfec_codec);
    for (uint32_t i = 0; i < nd; ++i) {
        nfec_codec* one = nullptr;
        const int rc = create_one(dev_at(i), kind, cfg->num_data, cfg->num_parity, cfg->vector_size, cfg->flags, &one);
        if (rc) return rc;  // the stripes built so far go with c
        c->stripes.emplace_back(one);
    }
    const nfec_codec* s0 = c->stripes[0].get();
    c->kind = kind;
    c->device = s0->device;
    c->opts = cfg->flags;
    c->k = s0->k;
    c->m = s0->m;
    c->vec = s0->vec;
    c->sym = s0->sym;
    c->cs = s0->cs;
    c->gen = s0->gen;
    c->async.device = s0->device;
    *out = c.release();
    return NFEC_OK;
}

int nfec_codec_num_devices(const nfec_codec* c, int32_t* devices, uint32_t cap)
{
    if (!c) return fail(NFEC_EINVAL, "null argument");
    const uint32_t n = c->stripes.empty() ? 1u : (uint32_t)c->stripes.size();
    for (uint32_t i = 0; i < n && devices && i < cap; ++i) devices[i] = c->stripes.empty() ? c->device : c->stripes[i]->device;
    return (int)n;
}

void nfec_codec_destroy(nfec_codec* codec) { delete codec; }

int nfec_build_generator(int kind, uint32_t num_data, uint32_t num_parity, void* host_out, size_t bytes)
{
    if (!host_out || num_data == 0 || num_parity == 0) return fail(NFEC_EINVAL, "bad argument");
    const size_t cnt = (size_t)num_data * num_parity;
    if (kind == NFEC_MDP) {
        if (num_data + num_parity > 255) return fail(NFEC_ERANGE, "MDP: numData + numParity > 255");
        if (bytes < cnt) return fail(NFEC_EINVAL, "output buffer too small");
        std::vector<uint8_t> g;
        mdp_generator_poly(num_parity, g);
        mdp_encode_matrix(g, num_parity, num_data, static_cast<uint8_t*>(host_out));
        return NFEC_OK;
    }
    if (kind != NFEC_RS8 && kind != NFEC_RS16) return fail(NFEC_EINVAL, "unknown codec kind");
    const size_t sym = kind == NFEC_RS16 ? 2 : 1;
    if (bytes < cnt * sym) return fail(NFEC_EINVAL, "output buffer too small");
    std::vector<uint32_t> rows;
    int rc = rs_generator(kind == NFEC_RS16 ? 16 : 8, num_data, num_parity, rows);
    if (rc) return fail(rc, "numData/numParity exceeds code limits");
    for (size_t i = 0; i < cnt; ++i) {
        if (sym == 2) static_cast<uint16_t*>(host_out)[i] = (uint16_t)rows[i];
        else static_cast<uint8_t*>(host_out)[i] = (uint8_t)rows[i];
    }
    return NFEC_OK;
}

int nfec_codec_get_info(const nfec_codec* c, nfec_codec_info* out)
{
    if (!c || !out) return fail(NFEC_EINVAL, "null argument");
    out->kind = c->kind;
    out->device = c->device;
    out->num_data = c->k;
    out->num_parity = c->m;
    out->vector_size = c->vec;
    out->symbol_bytes = c->sym;
    return NFEC_OK;
}

int nfec_codec_features(const nfec_codec* c)
{
    if (!c) return fail(NFEC_EINVAL, "null argument");
    const nfec_codec* p = primary(c);
    return (p->tmvp ? NFEC_FEATURE_RS16_TOEPLITZ : 0) | (p->tmvp_levels == 2 ? NFEC_FEATURE_RS16_TOEPLITZ2 : 0);
}

int nfec_codec_encode_paths(const nfec_codec* c, uint64_t* counts, uint32_t n)
{
    if (!c || (!counts && n)) return fail(NFEC_EINVAL, "null argument");
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t v = i < NFEC_PATH_COUNT ? c->enc_paths[i].load(std::memory_order_relaxed) : 0;
        for (const auto& st : c->stripes) v += i < NFEC_PATH_COUNT ? st->enc_paths[i].load(std::memory_order_relaxed) : 0;
        counts[i] = v;
    }
    return NFEC_PATH_COUNT;
}

int nfec_codec_decode_paths(const nfec_codec* c, uint64_t* counts, uint32_t n)
{
    if (!c || (!counts && n)) return fail(NFEC_EINVAL, "null argument");
    for (uint32_t i = 0; i < n; ++i) {
        uint64_t v = i < NFEC_DPATH_COUNT ? c->dec_paths[i].load(std::memory_order_relaxed) : 0;
        for (const auto& st : c->stripes) v += i < NFEC_DPATH_COUNT ? st->dec_paths[i].load(std::memory_order_relaxed) : 0;
        counts[i] = v;
    }
    return NFEC_DPATH_COUNT;
}

int nfec_codec_get_generator(const nfec_codec* c, void* host_out, size_t bytes)
{
    if (!c || !host_out) return fail(NFEC_EINVAL, "null argument");
    const size_t need = (size_t)c->m * c->k * c->sym;
    if (bytes < need) return fail(NFEC_EINVAL, "output buffer too small");
    for (size_t i = 0; i < (size_t)c->m * c->k; ++i) {
        if (c->sym == 2) static_cast<uint16_t*>(host_out)[i] = (uint16_t)c->gen[i];
        else static_cast<uint8_t*>(host_out)[i] = (uint8_t)c->gen[i];
    }
    return NFEC_OK;
}

int nfec_encode(nfec_codec* codec, const nfec_block_batch* batch, void* stream)
{
    int rc = check_batch(codec, batch);
    if (rc || batch->nblocks == 0) return rc;
    if (!(codec = stripe_for(codec, batch->blocks))) return fail(NFEC_EINVAL, "batch is not on a device of the codec");
    DeviceGuard g(codec->device);
    return encode_device(codec, batch, static_cast<hipStream_t>(stream));
}

int nfec_decode(nfec_codec* codec, const nfec_block_batch* batch, const uint16_t* erasure_locs,
                uint32_t erasure_stride, const uint16_t* erasure_counts, int32_t* status, void* stream)
{
    int rc = check_batch(codec, batch);
    if (rc || batch->nblocks == 0) return rc;
    if (erasure_stride == 0) return fail(NFEC_EINVAL, "erasure_stride must be > 0");
    if (!(codec = stripe_for(codec, batch->blocks))) return fail(NFEC_EINVAL, "batch is not on a device of the codec");
    DeviceGuard g(codec->device);
    return decode_device(codec, batch, erasure_locs, erasure_stride, erasure_counts, status,
                         static_cast<hipStream_t>(stream));
}

// ---- per-call NORM semantics (synchronous, host vectors) ----
// One call = gather the caller's vectors into the codec's pinned staging (host memcpy), one
// H2D copy, the kernels, one D2H copy of what the call writes, one synchronize, scatter.  The
// staging layout (device and pinned alike):
//   [0, 8)                 decode status (int32)
//   [8, 8 + meta)          decode erasure list (m uint16), count, numData
//   [data0, ...)           slots of round_up(vec, 8) bytes
// Per call this is latency-bound ("per-call drop-in"): NORM's block-at-once
// sites should use the batch calls instead.
namespace {

struct PerCall {
    uint8_t* dev;
    uint8_t* pin;
    uint32_t stride, data0;
};

int per_call_stage(nfec_codec* c, uint32_t nslots, PerCall& pc)
{
    pc.stride = round_up(c->vec, 8);
    pc.data0 = 8 + round_up((c->m + 2) * 2, 8);
    const size_t bytes = pc.data0 + (size_t)nslots * pc.stride;
    int rc = c->s_block.reserve(bytes);
    if (rc) return rc;
    if (c->s_pin_bytes < bytes) {
        if (c->s_pin) (void)hipHostFree(c->s_pin);
        c->s_pin = nullptr;
        c->s_pin_bytes = 0;
        if (hipHostMalloc(reinterpret_cast<void**>(&c->s_pin), bytes, hipHostMallocDefault) != hipSuccess)
            return fail(NFEC_ENOMEM, "per-call pinned staging allocation failed");
        c->s_pin_bytes = bytes;
    }
    if (!c->s_stream && hipStreamCreateWithFlags(&c->s_stream, hipStreamNonBlocking) != hipSuccess)
        return fail(NFEC_ENOMEM, "per-call stream creation failed");
    pc.dev = c->s_block.p;
    pc.pin = c->s_pin;
    return NFEC_OK;
}

}  // namespace

int nfec_encode_segment(nfec_codec* c, uint32_t segment_id, const void* data, void* const* parity)
{
    if (!c || !data || !parity) return fail(NFEC_EINVAL, "null argument");
    c = primary(c);
    if (c->host_only) return host_only_fail();
    if (segment_id >= c->k) return fail(NFEC_EINVAL, "segmentId >= numData");
    for (uint32_t i = 0; i < c->m; ++i)
        if (!parity[i]) return fail(NFEC_EINVAL, "null parity vector");
    DeviceGuard g(c->device);
    std::lock_guard<std::mutex> lk(c->mu);
    // slots: data, P0..P(m-1), and for MDP the new P(0..m-1) after them
    const uint32_t nslots = c->kind == NFEC_MDP ? 2 * c->m + 1 : c->m + 1;
    PerCall pc;
    int rc = per_call_stage(c, nslots, pc);
    if (rc) return rc;
    const hipStream_t st = c->s_stream;
    uint8_t* hp = pc.pin + pc.data0;
    // (measured: a kernel reading and writing the pinned staging directly, with no copies, is
    // slower per call -- 140 against 82 us for RS8(64,32): its loads cross PCIe one by one)
    uint8_t* d = pc.dev + pc.data0;
    std::memcpy(hp, data, c->vec);
    for (uint32_t i = 0; i < c->m; ++i) std::memcpy(hp + (size_t)(1 + i) * pc.stride, parity[i], c->vec);
    NFEC_HIP(hipMemcpyAsync(d, hp, (size_t)(c->m + 1) * pc.stride, hipMemcpyHostToDevice, st));
    uint32_t out_first = 1;
    if (c->kind == NFEC_RS8 || c->kind == NFEC_MDP) {
        Gf8MatmulArgs a;
        a.in_base = d;
        a.in_seg_stride = pc.stride;
        a.out_base = d;
        a.out_seg_stride = pc.stride;
        a.out_slot_mode = OUT_SLOT_AFTER_INPUT;
        a.rows_const = c->m;
        a.coef_col_stride = c->cs;
        a.vtab = c->d_vtab.p;
        a.nblocks = 1;
        a.vec_bytes = c->vec;
        if (c->kind == NFEC_RS8) {
            a.cols_const = 1;  // data in slot 0, column segment_id of the generator
            a.coef = c->d_coef.p + (size_t)segment_id * c->cs;
            a.accumulate = 1;  // parity[i] ^= G[k+i][segment_id] * data  (normEncoderRS8.cpp:473-483)
        } else {
            a.cols_const = c->m + 1;  // [d, P0..P(m-1)] -> new P in slots m+1..2m
            a.coef = c->d_mdp_step.p;
            out_first = c->m + 1;
        }
        if ((rc = launch_gf8_matmul(a, false, st))) return rc;
    } else {
        // the tower kernel over one column: the generator column segment_id is its own block
        // of the codec's table; parity slots 1..m, accumulated (normEncoderRS16.cpp:472-482).
        // A layout it does not take (its 2^31 offset bounds) goes to the exp-table kernel.
        Gf16T3Args t;
        t.base = d;
        t.block_stride = (uint64_t)(c->m + 1) * pc.stride;
        t.seg_stride = pc.stride;
        t.nblocks = 1;
        t.k = 1;
        t.m = c->m;
        t.vec_bytes = c->vec & ~1u;
        t.tw = c->tw ? c->d_twoff.p + (size_t)segment_id * 4u * c->m : nullptr;
        t.accumulate = 1;
        rc = c->tw && rs16_tw_full_covers(t) ? launch_rs16_tw_full(t, st) : NFEC_ENOTSUP;
        if (rc != NFEC_ENOTSUP && rc) return rc;
        if (rc == NFEC_ENOTSUP) {
            Gf16MatmulArgs a;
            a.in_base = d;
            a.in_seg_stride = pc.stride;
            a.cols_const = 1;
            a.out_base = d;
            a.out_seg_stride = pc.stride;
            a.out_slot_mode = OUT_SLOT_AFTER_INPUT;
            a.rows_const = c->m;
            a.coef = reinterpret_cast<const uint16_t*>(c->d_coef.p) + (size_t)segment_id * c->cs;
            a.coef_col_stride = c->cs;
            a.exp_tab = reinterpret_cast<const uint16_t*>(c->d_exp.p);
            a.log_tab = c->d_log.p;
            a.nblocks = 1;
            a.vec_bytes = c->vec & ~1u;
            a.accumulate = 1;
            if ((rc = launch_gf16_matmul(a, st))) return rc;
        }
    }
    const size_t off = (size_t)out_first * pc.stride;
    NFEC_HIP(hipMemcpyAsync(hp + off, d + off, (size_t)c->m * pc.stride, hipMemcpyDeviceToHost, st));
    NFEC_HIP(hipStreamSynchronize(st));
    // RS16 never writes an odd last byte: it came back unchanged from the upload
    for (uint32_t i = 0; i < c->m; ++i) std::memcpy(parity[i], hp + off + (size_t)i * pc.stride, c->vec);
    return NFEC_OK;
}

int nfec_encode_segment_host(nfec_codec* c, uint32_t segment_id, const void* data, void* const* parity)
{
    if (!c || !data || !parity) return fail(NFEC_EINVAL, "null argument");
    c = primary(c);  // a multi-device codec: the first stripe holds the host tables (mdp_g)
    if (segment_id >= c->k) return fail(NFEC_EINVAL, "segmentId >= numData");
    for (uint32_t i = 0; i < c->m; ++i)
        if (!parity[i]) return fail(NFEC_EINVAL, "null parity vector");
    const uint8_t* d = static_cast<const uint8_t*>(data);
    const int isa = host_gf8_isa();
    if (c->kind == NFEC_RS16) {
        // vec / 2 native-endian symbols; an odd last byte is never touched (normEncoderRS16.cpp:479)
        host_gf16_addmul_rows(reinterpret_cast<uint16_t* const*>(parity), static_cast<const uint16_t*>(data),
                              c->gen.data() + segment_id, c->k, c->m, c->vec / 2, isa);
        return NFEC_OK;
    }
    if (c->kind == NFEC_MDP) {
        // the reference's LFSR step: s = data ^ P0 (its scratch copy of P0), then the shift
        host_mdp_step(reinterpret_cast<uint8_t* const*>(parity), d, c->mdp_g.data(), c->m, c->vec, isa);
        return NFEC_OK;
    }
    host_gf8_addmul_rows(reinterpret_cast<uint8_t* const*>(parity), d, c->gen.data() + segment_id, c->k, c->m, c->vec,
                         isa);
    return NFEC_OK;
}

namespace {
unsigned host_copy_threads();
}

// The host repair's products: dst[r] (^)= sum_j coef[r][j] * srcs[j] over nelem bytes (GF(2^8))
// or symbols (GF(2^16)), row dot products over pieces of the vectors, so a piece of every column
// stays in cache while all rows take it; a repair of more than 8 MiB of products splits the
// vectors over host threads (disjoint element ranges, no sharing).
static int host_rows_apply(bool wide, void* const* dst, uint32_t nrows, const void* const* srcs, uint32_t ncol,
                           const uint16_t* coef, size_t nelem, bool acc)
{
    const int isa = host_gf8_isa();
    const uint64_t work = (uint64_t)nrows * ncol * nelem * (wide ? 2 : 1);
    const size_t piece = wide ? 1024 : 2048;
    auto run = [&](size_t e0, size_t e1) {
        for (size_t c0 = e0; c0 < e1; c0 += piece) {
            const size_t len = std::min(piece, e1 - c0);
            for (uint32_t r = 0; r < nrows; ++r) {
                if (!dst[r]) continue;
                if (wide)
                    host_gf16_dot(static_cast<uint16_t*>(dst[r]) + c0, reinterpret_cast<const uint16_t* const*>(srcs), c0,
                                  coef + (size_t)r * ncol, ncol, len, acc, isa);
                else
                    host_gf8_dot(static_cast<uint8_t*>(dst[r]) + c0, reinterpret_cast<const uint8_t* const*>(srcs), c0,
                                 coef + (size_t)r * ncol, ncol, len, acc, isa);
            }
        }
    };
    const unsigned nt = work > (8ull << 20)
                            ? (unsigned)std::min<uint64_t>(std::min<uint64_t>(host_copy_threads(), work >> 22), nelem / 256)
                            : 1u;
    if (nt <= 1) {
        run(0, nelem);
        return NFEC_OK;
    }
    // ranges in multiples of 128 elements, on the process's host pool
    const size_t per = ((nelem + nt - 1) / nt + 127) & ~(size_t)127;
    return host_parallel_for(nt, [&](unsigned t) {
        const size_t e0 = std::min(nelem, t * per), e1 = std::min(nelem, e0 + per);
        if (e0 < e1) run(e0, e1);
    });
}

// MDP one-block repair on the host: the closed-form Forney map of mdp_plan_kernel
// (kernels_plan.hip; tests/test_mdp_algebra.py), C[r][v] = [Dinv_r beta_r^m] [gamma_v^(m+1)
// Lambda(1 / gamma_v)] / (gamma_v beta_r + 1) over the surviving slots v, written over the erased
// source (the reference's syndrome decode, normEncoderMDP.cpp:333-430, reads erased source as
// zeros and missing parity as absent).  The list is already validated and es > 0.
static int mdp_decode_host(const nfec_codec* c, void* const* vectors, uint32_t nd, uint32_t ec,
                            const uint32_t* locs, uint32_t es)
{
    const Field& f = gf8();
    const uint32_t m = c->m, nvecs = nd + m, deg = 2 * m;
    auto mul = [&](uint32_t x, uint32_t y) -> uint32_t { return (x && y) ? f.exp[f.log[x] + f.log[y]] : 0u; };
    // erasure locator lambda(x) = prod_i (1 + X_i x), X_i = alpha^(nvecs-1-loc_i)
    std::vector<uint32_t> lam(deg, 0);
    lam[0] = 1;
    for (uint32_t i = 0; i < ec; ++i) {
        const uint32_t X = f.exp[nvecs - 1 - locs[i]];
        for (uint32_t j = deg - 1; j > 0; --j) lam[j] ^= mul(X, lam[j - 1]);
    }
    // row factors log(Dinv_r beta_r^m), log beta_r
    std::vector<uint32_t> lrow(es), lbeta(es);
    for (uint32_t r = 0; r < es; ++r) {
        const uint32_t lb = (255u - (nvecs - 1 - locs[r])) % 255u;
        uint32_t denom = 0;
        for (uint32_t j = 1; j < deg; j += 2)
            if (lam[j]) denom ^= f.exp[(f.log[lam[j]] + (uint64_t)lb * (j - 1)) % 255u];
        const uint32_t ldinv = denom ? (255u - f.log[denom]) % 255u : 0u;  // GINV[0] = 1 (galois.cpp:39)
        lbeta[r] = lb;
        lrow[r] = (ldinv + (m % 255u) * lb) % 255u;
    }
    std::vector<uint8_t> erased(nvecs, 0);
    for (uint32_t i = 0; i < ec; ++i) erased[locs[i]] = 1;
    std::vector<const void*> srcs;
    std::vector<uint32_t> lcols, lgams;
    for (uint32_t v = 0; v < nvecs; ++v) {
        if (erased[v] || !vectors[v]) continue;  // a NULL survivor reads as zeros, as on the GPU
        const uint32_t lgam = (nvecs - 1 - v) % 255u, step = (255u - lgam) % 255u;
        uint32_t acc = 0;
        for (uint32_t i = 0, pi = 0; i <= ec; ++i, pi = (pi + step) % 255u)
            if (lam[i]) acc ^= f.exp[f.log[lam[i]] + pi];
        srcs.push_back(vectors[v]);
        lcols.push_back(((m + 1u) % 255u * lgam + f.log[acc]) % 255u);  // acc != 0: v survived
        lgams.push_back(lgam);
    }
    const uint32_t ncol = (uint32_t)srcs.size();
    std::vector<uint16_t> coef((size_t)es * ncol);
    std::vector<void*> dst(es);
    for (uint32_t r = 0; r < es; ++r) {
        dst[r] = vectors[locs[r]];
        for (uint32_t j = 0; j < ncol; ++j) {
            const uint32_t w1 = f.exp[lgams[j] + lbeta[r]] ^ 1u;  // gamma_v beta_r + 1, nonzero
            coef[(size_t)r * ncol + j] = (uint16_t)f.exp[(lrow[r] + lcols[j] + 255u - f.log[w1]) % 255u];
        }
    }
    return host_rows_apply(false, dst.data(), es, srcs.data(), ncol, coef.data(), c->vec, false);
}

int nfec_decode_vectors_host(nfec_codec* c, void* const* vectors, uint32_t num_data, uint32_t erasure_count,
                             const uint32_t* erasure_locs)
{
    if (!c || !vectors || (erasure_count && !erasure_locs)) return fail(NFEC_EINVAL, "null argument");
    c = primary(c);
    if (c->kind != NFEC_MDP && c->h_lwp.empty())
        return fail(NFEC_ENOTSUP, "host decode: the codec has no closed-form plan constants");
    if (num_data == 0 || num_data > c->k) return fail(NFEC_EINVAL, "numData out of range");
    const uint32_t k = c->k, m = c->m, nd = num_data;
    // the reference's undefined cases (more erasures than parity, unsorted or out-of-range lists)
    // leave the block alone and return 0, as the GPU plans do
    if (erasure_count > m) return 0;
    uint32_t es = 0;
    for (uint32_t i = 0; i < erasure_count; ++i) {
        if (erasure_locs[i] >= nd + m || (i && erasure_locs[i] <= erasure_locs[i - 1])) return 0;
        es += erasure_locs[i] < nd;
    }
    if (es == 0) return (int)erasure_count;  // only parity lost: nothing is filled (:732)
    if (c->kind == NFEC_MDP) {
        const int rc = mdp_decode_host(c, vectors, nd, erasure_count, erasure_locs, es);
        return rc ? rc : (int)erasure_count;
    }
    const bool wide = c->kind == NFEC_RS16;
    const Field& f = wide ? gf16() : gf8();
    const int64_t q = f.q;
    auto md = [&](int64_t v) { v %= q; return v < 0 ? v + q : v; };
    auto L = [&](uint32_t v) { return (int64_t)f.log[v]; };
    // substitute parities: the first es surviving ones in slot order (normEncoderRS8.cpp:689-711)
    std::vector<uint32_t> par;
    {
        uint32_t i = es;  // the parity entries of the sorted list follow the source ones
        for (uint32_t p = 0; p < m && par.size() < es; ++p) {
            if (i < erasure_count && erasure_locs[i] == nd + p) {
                ++i;
                continue;
            }
            par.push_back(p);
        }
        if (par.size() < es) return 0;  // not enough parity
    }
    std::vector<uint32_t> xs(es), yt(es);
    std::vector<uint8_t> erased(nd, 0);
    for (uint32_t s = 0; s < es; ++s) {
        xs[s] = rs_point(f, erasure_locs[s]);
        yt[s] = rs_point(f, k + par[s]);
        erased[erasure_locs[s]] = 1;
    }
    // A^-1[s][t] = exp(lA[s] + lB[t] - log(x_s + y_t)); the map of a received source column j is
    // exp(lA[s] + lC[j] - log(x_s + x_j)) (rs8_plan_rt_kernel's algebra, tests/test_rt_algebra.py)
    std::vector<int64_t> lA(es), lB(es);
    for (uint32_t s = 0; s < es; ++s) {
        int64_t a = c->h_lwp[erasure_locs[s]], b = -(int64_t)c->h_lw[par[s]];
        for (uint32_t t = 0; t < es; ++t) {
            a += L(xs[s] ^ yt[t]);
            b += L(yt[s] ^ xs[t]);
            if (t != s) a -= L(xs[s] ^ xs[t]), b -= L(yt[s] ^ yt[t]);
        }
        lA[s] = md(a);
        lB[s] = md(b);
    }
    // columns: the surviving (non-NULL) source, then the substitute parities (a NULL parity reads
    // as zeros, as in the GPU path)
    std::vector<const void*> srcs;
    std::vector<int64_t> lcol;   // log factor per column
    std::vector<uint32_t> pts;   // its point
    for (uint32_t j = 0; j < nd; ++j) {
        if (erased[j] || !vectors[j]) continue;
        const uint32_t xj = rs_point(f, j);
        int64_t lc = -(int64_t)c->h_lwp[j];
        for (uint32_t t = 0; t < es; ++t) lc += L(xj ^ xs[t]) - L(xj ^ yt[t]);
        srcs.push_back(vectors[j]);
        lcol.push_back(md(lc));
        pts.push_back(xj);
    }
    for (uint32_t t = 0; t < es; ++t) {
        if (!vectors[nd + par[t]]) continue;
        srcs.push_back(vectors[nd + par[t]]);
        lcol.push_back(lB[t]);
        pts.push_back(yt[t]);
    }
    const uint32_t ncol = (uint32_t)srcs.size();
    std::vector<uint16_t> coef((size_t)es * ncol);
    std::vector<void*> dst(es);
    for (uint32_t s = 0; s < es; ++s) {
        dst[s] = vectors[erasure_locs[s]];
        for (uint32_t j = 0; j < ncol; ++j)
            coef[(size_t)s * ncol + j] = (uint16_t)f.exp[md(lA[s] + lcol[j] - L(xs[s] ^ pts[j]))];
    }
    // RS16: an odd last byte is never touched
    const int rc = host_rows_apply(wide, dst.data(), es, srcs.data(), ncol, coef.data(), wide ? c->vec / 2 : c->vec, true);
    return rc ? rc : (int)erasure_count;
}

// Repair products up to which one-block Decode stays on the host, from tools/percall
// (profiles/r04/percall.jsonl): the host path (row dot products, 8 threads past 8 MiB) beat the
// GPU round trip at every measured size -- RS8(128,127) x 8192 B with 100 erasures (105 MB of
// products) 0.36 against 0.79 ms, MDP (209 MB) 0.42 against 0.99 ms, RS16(400,100) with 50
// erasures (14 M symbol products) 0.31 against 0.86 ms -- so the bounds sit a few times past them.
static constexpr uint64_t kHostDecodeRs8Bytes = 256ull << 20;
static constexpr uint64_t kHostDecodeMdpBytes = 512ull << 20;
static constexpr uint64_t kHostDecodeRs16Symbols = 64ull << 20;

int nfec_decode_host_preferred(const nfec_codec* c, uint32_t num_data, uint32_t erasure_count)
{
    if (!c) return 0;
    c = primary(c);
    if (c->host_only) return c->kind == NFEC_MDP || !c->h_lwp.empty() ? 1 : 0;
    const uint64_t e = std::min(erasure_count, c->m);
    // products of the repair: erased rows x columns read x symbols
    if (c->kind == NFEC_MDP) return e * (num_data + c->m) * c->vec <= kHostDecodeMdpBytes ? 1 : 0;
    if (c->h_lwp.empty()) return 0;
    if (c->kind == NFEC_RS8) return e * num_data * c->vec <= kHostDecodeRs8Bytes ? 1 : 0;
    return e * num_data * (c->vec / 2) <= kHostDecodeRs16Symbols ? 1 : 0;
}

int nfec_decode_vectors(nfec_codec* c, void* const* vectors, uint32_t num_data, uint32_t erasure_count,
                        const uint32_t* erasure_locs)
{
    if (!c || !vectors || (erasure_count && !erasure_locs)) return fail(NFEC_EINVAL, "null argument");
    c = primary(c);
    if (c->host_only) return host_only_fail();
    if (num_data == 0 || num_data > c->k) return fail(NFEC_EINVAL, "numData out of range");
    if (erasure_count > c->m) return 0;
    DeviceGuard g(c->device);
    const uint32_t nslots = num_data + c->m;
    // the whole call runs under mu: the staging and the decode workspace are the codec's
    std::lock_guard<std::mutex> lk(c->mu);
    PerCall pc;
    int rc = per_call_stage(c, c->k + c->m, pc);
    if (rc) return rc;
    const hipStream_t st = c->s_stream;
    uint16_t* hl = reinterpret_cast<uint16_t*>(pc.pin + 8);
    std::memset(hl, 0, pc.data0 - 8);
    for (uint32_t i = 0; i < erasure_count; ++i) hl[i] = (uint16_t)erasure_locs[i];
    hl[c->m] = (uint16_t)erasure_count;
    hl[c->m + 1] = (uint16_t)num_data;
    // gather: present vectors as given (erased source arrives zero-filled, normObject.cpp:1579),
    // missing (NULL) parity as zeros
    uint8_t* hp = pc.pin + pc.data0;
    for (uint32_t s = 0; s < nslots; ++s) {
        if (vectors[s]) std::memcpy(hp + (size_t)s * pc.stride, vectors[s], c->vec);
        else std::memset(hp + (size_t)s * pc.stride, 0, c->vec);
    }
    NFEC_HIP(hipMemcpyAsync(pc.dev + 8, pc.pin + 8, pc.data0 - 8 + (size_t)nslots * pc.stride, hipMemcpyHostToDevice, st));
    uint16_t* dl = reinterpret_cast<uint16_t*>(pc.dev + 8);
    int32_t* dstatus = reinterpret_cast<int32_t*>(pc.dev);
    // The reference XORs the repair into the erased buffers (accumulate).  NORM hands them in
    // zero-filled (normObject.cpp:1579), and then overwriting is the same; a full block
    // (numData = k) with zero erased buffers therefore takes the batch fast paths (fused RS8
    // repair, RS16 stages on the tower kernel), anything else the general ones.
    bool zero_erased = true;
    for (uint32_t i = 0; i < erasure_count && zero_erased; ++i) {
        const uint32_t s = erasure_locs[i];
        if (s >= num_data || !vectors[s]) continue;
        const uint8_t* v = static_cast<const uint8_t*>(vectors[s]);
        uint64_t acc = 0, w;
        size_t j = 0;
        for (; j + 8 <= c->vec; j += 8) {
            std::memcpy(&w, v + j, 8);
            acc |= w;
        }
        for (; j < c->vec; ++j) acc |= v[j];
        zero_erased = acc == 0;
    }
    nfec_block_batch b{};
    b.blocks = pc.dev + pc.data0;
    b.block_stride = (uint64_t)(c->k + c->m) * pc.stride;
    b.seg_stride = pc.stride;
    b.nblocks = 1;
    b.num_data = num_data == c->k ? nullptr : dl + c->m + 1;
    b.flags = (c->kind == NFEC_MDP || zero_erased) ? 0 : NFEC_ACCUMULATE;
    if ((rc = decode_device(c, &b, dl, c->m, dl + c->m, dstatus, st, true))) return rc;
    // status and the source slots in one copy (the meta bytes between them ride along)
    NFEC_HIP(hipMemcpyAsync(pc.pin, pc.dev, pc.data0 + (size_t)num_data * pc.stride, hipMemcpyDeviceToHost, st));
    NFEC_HIP(hipStreamSynchronize(st));
    int32_t status;
    std::memcpy(&status, pc.pin, sizeof(status));
    if (status > 0) {
        const size_t out_bytes = c->sym == 2 ? (c->vec & ~1u) : c->vec;  // RS16: odd last byte untouched
        for (uint32_t i = 0; i < erasure_count; ++i) {
            const uint32_t s = erasure_locs[i];
            if (s >= num_data) break;  // parity is never filled (normEncoderRS8.cpp:732)
            if (vectors[s]) std::memcpy(vectors[s], hp + (size_t)s * pc.stride, out_bytes);
        }
    }
    return status;
}

// ---- host-resident batches: pinned staging, H2D || compute || D2H over two slots ----
// Host-resident batches: a pipeline of device slots, each on its own stream, with the H2D
// copy, the kernels and the D2H copy of chunk i overlapping chunk i+1's.  Only the bytes the
// operation reads are uploaded and only the bytes it writes are downloaded:
//   encode  (unshortened, overwrite): up source slots [0,k), down parity slots [k,k+m)
//   encode  (shortened or accumulate): up/down the whole block span
//   decode: up the whole block span, down source slots [0,k) (unerased bytes come back
//           unchanged; parity slots are never written).
// A pinned (page-locked / hipHostRegister'ed) caller buffer is DMA'd directly; a pageable one
// goes through pinned staging with the copy split over host threads.
namespace {

bool host_is_pinned(const void* p)
{
    hipPointerAttribute_t at;
    std::memset(&at, 0, sizeof(at));
    const hipError_t e = hipPointerGetAttributes(&at, p);
    if (e != hipSuccess) {
        (void)hipGetLastError();
        return false;
    }
    return at.type == hipMemoryTypeHost;
}

// the device's address of pinned host memory (kernels read and write it over PCIe), or null
uint8_t* host_device_ptr(const void* p)
{
    hipPointerAttribute_t at;
    std::memset(&at, 0, sizeof(at));
    if (hipPointerGetAttributes(&at, p) != hipSuccess || at.type != hipMemoryTypeHost) {
        (void)hipGetLastError();
        return nullptr;
    }
    return static_cast<uint8_t*>(at.devicePointer);
}

// pieces one host copy is cut into (at least 4 MiB each): as many as the process's host pool
// has workers, which every concurrent call (and stripe) shares
unsigned host_copy_threads() { return host_pool_size(); }

// rows x width bytes, strided on both sides, split over host threads for large copies
int copy2d(uint8_t* dst, uint64_t dpitch, const uint8_t* src, uint64_t spitch, uint64_t width, uint32_t rows)
{
    if (rows == 0 || width == 0) return NFEC_OK;
    auto run = [=](uint32_t r0, uint32_t r1) {
        if (dpitch == width && spitch == width) {
            std::memcpy(dst + r0 * width, src + r0 * width, (size_t)(r1 - r0) * width);
            return;
        }
        for (uint32_t r = r0; r < r1; ++r) std::memcpy(dst + r * dpitch, src + r * spitch, (size_t)width);
    };
    const uint64_t bytes = width * rows;
    const unsigned nt = (unsigned)std::min<uint64_t>(std::min<uint64_t>(host_copy_threads(), rows),
                                                      std::max<uint64_t>(1, bytes >> 22));
    if (nt <= 1) {
        run(0, rows);
        return NFEC_OK;
    }
    const uint32_t per = (rows + nt - 1) / nt;
    return host_parallel_for(nt, [&](unsigned t) {
        const uint32_t r0 = std::min<uint32_t>(rows, t * per), r1 = std::min<uint32_t>(rows, r0 + per);
        if (r0 < r1) run(r0, r1);
    });
}

}  // namespace

// ---- cached host staging ----
// The pipelines' device slots, pinned staging, streams and events live in the codec and grow
// on demand: allocating (and freeing, which synchronises the whole device) per call would
// stall every other codec's work on the GPU -- two codecs driven from two host threads (the
// mixed RS8/RS16 stream of BASELINE C5) would serialise.  Host-batch calls on one codec are
// serialised by the codec's stage_mu (the reference's codec instances are single-threaded,
// normApi.cpp:55,126; here concurrent callers of one codec wait rather than race).
static int grow_dev(void** p, size_t& cap, size_t need)
{
    if (cap >= need) return NFEC_OK;
    if (*p) (void)hipFree(*p);
    *p = nullptr;
    cap = 0;
    if (hipMalloc(p, need) != hipSuccess) return fail(NFEC_ENOMEM, "staging allocation failed");
    cap = need;
    return NFEC_OK;
}

static int grow_pin(void** p, size_t& cap, size_t need)
{
    if (cap >= need) return NFEC_OK;
    if (*p) (void)hipHostFree(*p);
    *p = nullptr;
    cap = 0;
    if (hipHostMalloc(p, need, hipHostMallocDefault) != hipSuccess) return fail(NFEC_ENOMEM, "pinned staging allocation failed");
    cap = need;
    return NFEC_OK;
}

static int stage_slot(nfec_codec* c, uint32_t i, size_t dev_bytes, size_t pin_bytes, size_t meta_bytes,
                      size_t stat_bytes, HostSlot*& out)
{
    HostSlot& s = c->stage.slot[i];
    int rc;
    const uint8_t* pin_before = s.pin;
    if ((rc = grow_dev(reinterpret_cast<void**>(&s.dev), s.dev_bytes, dev_bytes)) ||
        (pin_bytes && (rc = grow_pin(reinterpret_cast<void**>(&s.pin), s.pin_bytes, pin_bytes))) ||
        (rc = grow_dev(reinterpret_cast<void**>(&s.dmeta), s.meta_bytes, meta_bytes)) ||
        (rc = grow_pin(reinterpret_cast<void**>(&s.hmeta), s.hmeta_bytes, meta_bytes)) ||
        (rc = grow_dev(reinterpret_cast<void**>(&s.dstat), s.dstat_bytes, stat_bytes)) ||
        (rc = grow_pin(reinterpret_cast<void**>(&s.hstat), s.hstat_bytes, stat_bytes)))
        return rc;
    if (s.pin != pin_before) s.pin_dev = s.pin ? host_device_ptr(s.pin) : nullptr;
    if (!s.st) {
        const hipError_t se = hipStreamCreateWithFlags(&s.st, hipStreamNonBlocking);
        if (se != hipSuccess ||
            hipEventCreateWithFlags(&s.done, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.ev_up, hipEventDisableTiming) != hipSuccess ||
            hipEventCreateWithFlags(&s.ev_cd, hipEventDisableTiming) != hipSuccess)
            return fail(NFEC_ENOMEM, "staging stream creation failed");
    }
    if (!c->stage.cst) {
        // the decode kernels run at the highest stream priority: the slot moves of the other
        // chunks are PCIe-bound and must not hold the CUs the compute waits for
        int least = 0, greatest = 0;
        if (hipDeviceGetStreamPriorityRange(&least, &greatest) != hipSuccess) {
            (void)hipGetLastError();
            greatest = 0;
        }
        if (hipStreamCreateWithPriority(&c->stage.cst, hipStreamNonBlocking, greatest) != hipSuccess)
            return fail(NFEC_ENOMEM, "staging stream creation failed");
    }
    out = &s;
    return NFEC_OK;
}

// Per-chunk metadata (numData, erasure lists, counts) goes up through the slot's pinned mirror:
// an async copy straight from the caller's pageable arrays is staged by the runtime and
// blocks the host thread until the link drains, which stalls the pipeline behind the other
// chunks' transfers.  (The slot is reused only after its previous chunk completed.)
static hipError_t meta_up(HostSlot& s, uint16_t* dev, const uint16_t* src, size_t count)
{
    const size_t off = reinterpret_cast<uint8_t*>(dev) - reinterpret_cast<uint8_t*>(s.dmeta);
    std::memcpy(s.hmeta + off, src, count * 2);
    return hipMemcpyAsync(dev, s.hmeta + off, count * 2, hipMemcpyHostToDevice, s.st);
}

// Blocks per pipeline chunk: about 128 MiB (RS8(64,32) x 1400 B, 65,536 pinned blocks: 1,024-block
// chunks 22.98 GiB/s, 2,048 22.7, 4,096 22.55, 512 21.68 on one box), but never fewer than the blocks it takes to fill
// the GPU when the kernels run one wave per block (RS16, MDP, the generic RS8 kernels: 16 waves
// per CU, 4096 blocks), and at most 4 GiB per slot.
static uint32_t host_chunk(const nfec_codec* c, uint64_t dbs, uint32_t nblocks)
{
    if (const char* e = std::getenv("NFEC_HOST_CHUNK_BLOCKS"))  // tests: force multi-chunk pipelines
        if (std::atol(e) > 0) return (uint32_t)std::min<uint64_t>((uint64_t)std::atol(e), nblocks);
    const bool per_block = !(c->kind == NFEC_RS8 && has_bitsliced(c->k, c->m));
    uint64_t ch = std::max<uint64_t>(1, (128ull << 20) / std::max<uint64_t>(dbs, 1));
    if (per_block) ch = std::max<uint64_t>(ch, 4096);
    ch = std::min<uint64_t>(ch, std::max<uint64_t>(1, (4ull << 30) / std::max<uint64_t>(dbs, 1)));
    return (uint32_t)std::min<uint64_t>(ch, nblocks);
}

static void stage_drain(nfec_codec* c)
{
    for (auto& s : c->stage.slot)
        if (s.st) (void)hipStreamSynchronize(s.st);
    if (c->stage.cst) (void)hipStreamSynchronize(c->stage.cst);
}

// The codec's decode workspace (plan, z rows, inverses) is shared by all of its decode calls,
// so the host pipelines run every chunk's decode on one compute stream: slot stream upload ->
// event -> compute-stream decode -> event -> slot stream download.  (Encode reads only the
// codec's constants and runs on the slot streams.)
// Blocks whose numData (known on the host) equals k go to the unshortened fast kernels in
// sub-batches of their own; only the others carry their numData.  NORM batches are mostly full
// blocks with one short block ending each object, and one short block would otherwise send the
// whole batch down the generic (numData-aware) kernels.  Full runs shorter than kMinFullRun stay
// with their neighbours: a launch per handful of blocks costs more than it saves.
extern "C++" template <typename F>
static int split_full_runs(const uint16_t* hnd, uint32_t n, uint32_t k, F launch)
{
    constexpr uint32_t kMinFullRun = 32;
    if (!hnd) return launch(0u, n, false);
    uint32_t i = 0;
    while (i < n) {
        uint32_t rs = n, re = n;
        for (uint32_t j = i; j < n;) {
            if (hnd[j] != k) {
                ++j;
                continue;
            }
            uint32_t e = j;
            while (e < n && hnd[e] == k) ++e;
            if (e - j >= kMinFullRun) {
                rs = j;
                re = e;
                break;
            }
            j = e;
        }
        int rc;
        if (rs > i && (rc = launch(i, rs - i, true))) return rc;
        if (rs < n && (rc = launch(rs, re - rs, false))) return rc;
        i = re;
    }
    return NFEC_OK;
}

static int decode_serialized(nfec_codec* c, const nfec_block_batch* db, const uint16_t* dl, uint32_t lstride,
                             const uint16_t* dc, HostSlot& s, uint32_t status_off = 0)
{
    NFEC_HIP(hipEventRecord(s.ev_up, s.st));
    NFEC_HIP(hipStreamWaitEvent(c->stage.cst, s.ev_up, 0));
    const int rc = decode_device(c, db, dl, lstride, dc, s.dstat + status_off, c->stage.cst);
    if (rc) return rc;
    NFEC_HIP(hipEventRecord(s.ev_cd, c->stage.cst));
    NFEC_HIP(hipStreamWaitEvent(s.st, s.ev_cd, 0));
    return NFEC_OK;
}

// One chunk of a host-resident decode with zero-copy slot moves (run_host_batch): metadata up
// by DMA, the read slots gathered from host memory by a kernel (hdev: the caller's pinned
// blocks as the device addresses them; null: a pageable caller, whose chunk is first copied
// into the slot's pinned staging by host threads), the decode on the compute stream, the
// repaired slots scattered back by a kernel, the status by DMA.  Ends with s.done recorded.
static int host_decode_zc(nfec_codec* c, const nfec_block_batch* hb, HostSlot& s, uint32_t b0, uint32_t nb,
                          uint32_t chunk, const uint16_t* locs, uint32_t lstride, const uint16_t* counts,
                          uint8_t* hdev, uint64_t ul)
{
    const uint64_t hbs = hb->block_stride, ss = hb->seg_stride;
    const uint64_t dbs = (uint64_t)(c->k + c->m) * ss;
    uint8_t* hsrc = static_cast<uint8_t*>(hb->blocks) + (uint64_t)b0 * hbs;
    uint16_t* dnd = hb->num_data ? s.dmeta : nullptr;
    uint16_t* dlocs = s.dmeta + chunk;
    uint16_t* dcnt = dlocs + (size_t)chunk * lstride;
    hipError_t ae = meta_up(s, dlocs, locs + (uint64_t)b0 * lstride, (size_t)nb * lstride);
    if (ae == hipSuccess) ae = meta_up(s, dcnt, counts + b0, nb);
    if (ae == hipSuccess && dnd)
        ae = meta_up(s, dnd, hb->num_data + b0, nb);
    if (ae != hipSuccess) return hip_fail(ae, "host decode metadata upload");
    SlotMoveArgs mv;
    if (hdev) {
        mv.src = hdev + (uint64_t)b0 * hbs;
        mv.src_block_stride = hbs;
    } else {
        if (!s.pin_dev) return fail(NFEC_EDEVICE, "pinned staging is not device-mapped");
        if (const int rc = copy2d(s.pin, dbs, hsrc, hbs, ul, nb)) return rc;
        mv.src = s.pin_dev;
        mv.src_block_stride = dbs;
    }
    mv.src_seg_stride = (uint32_t)ss;
    mv.dst = s.dev;
    mv.dst_block_stride = dbs;
    mv.dst_seg_stride = (uint32_t)ss;
    mv.nblocks = nb;
    mv.k = c->k;
    mv.m = c->m;
    mv.bytes = c->vec;
    mv.num_data = dnd;
    mv.locs = dlocs;
    mv.lstride = lstride;
    mv.counts = dcnt;
    mv.mode = c->kind == NFEC_MDP ? SLOTS_ALL_IN : SLOTS_RS_IN;
    mv.accumulate = (hb->flags & NFEC_ACCUMULATE) ? 1u : 0u;
    int rc = launch_slot_move(mv, s.st);
    if (rc) return rc;
    nfec_block_batch db = *hb;
    db.blocks = s.dev;
    db.block_stride = dbs;
    db.nblocks = nb;
    db.num_data = dnd;
    // timing probes (diagnostic library): 1 no decode, 2 no scatter, 3 neither.  Measured (16k
    // blocks RS8(64,32), tools/host_rate.py): 33.1 / 29.3 / 29.9 / 29.1 ms; a window DMA for the
    // download instead of the scatter: 51 ms (DMA writes and zero-copy reads share the link badly)
    static const long probe = diag_knob("NFEC_ZC_PROBE", 0, 0, 3);
    if (!(probe & 1)) rc = split_full_runs(hb->num_data ? hb->num_data + b0 : nullptr, nb, c->k, [&](uint32_t o, uint32_t n, bool nd) {
        nfec_block_batch sb = db;
        sb.blocks = s.dev + o * dbs;
        sb.nblocks = n;
        sb.num_data = nd ? dnd + o : nullptr;
        return decode_serialized(c, &sb, dlocs + (uint64_t)o * lstride, lstride, dcnt + o, s, o);
    });
    if (rc) return rc;
    // repaired source slots back (RS16 never writes an odd last byte, normEncoderRS16.cpp:733)
    SlotMoveArgs out = mv;
    out.src = s.dev;
    out.src_block_stride = dbs;
    out.dst = hdev ? hdev + (uint64_t)b0 * hbs : s.pin_dev;
    out.dst_block_stride = hdev ? hbs : dbs;
    out.bytes = c->sym == 2 ? (c->vec & ~1u) : c->vec;
    out.status = s.dstat;
    out.mode = SLOTS_OUT;
    if (!(probe & 2) && (rc = launch_slot_move(out, s.st))) return rc;
    ae = hipMemcpyAsync(s.hstat, s.dstat, (size_t)nb * 4, hipMemcpyDeviceToHost, s.st);
    if (ae == hipSuccess) ae = hipEventRecord(s.done, s.st);
    return ae == hipSuccess ? NFEC_OK : hip_fail(ae, "host decode status");
}

// A host batch on a codec over several devices: contiguous block ranges [i*B/N, (i+1)*B/N), one
// per stripe, each through that stripe's own pipeline on a host thread of its own (SURVEY 8e:
// no exchange between the ranges).  fn(stripe, first block, blocks) runs one range.  The
// first failing range's status and message are returned on the calling thread.
extern "C++" template <typename F>
static int run_striped(nfec_codec* c, uint32_t nblocks, F fn)
{
    const uint32_t ns = (uint32_t)std::min<size_t>(c->stripes.size(), std::max(nblocks, 1u));
    std::vector<int> rcs(ns, NFEC_OK);
    std::vector<std::string> errs(ns);
    auto one = [&](uint32_t i) {
        const uint32_t lo = (uint32_t)((uint64_t)nblocks * i / ns), hi = (uint32_t)((uint64_t)nblocks * (i + 1) / ns);
        rcs[i] = hi > lo ? fn(c->stripes[i].get(), lo, hi - lo) : NFEC_OK;
        if (rcs[i] < 0) errs[i] = last_error_cstr();
    };
    // one driver thread per stripe (they mostly wait on their GPU; the copies go to the host pool)
    std::vector<std::thread> th;
    std::vector<uint32_t> inline_ranges;
    for (uint32_t i = 1; i < ns; ++i) {
        try {
            th.emplace_back(one, i);
        } catch (...) {
            inline_ranges.push_back(i);  // no thread to be had: that range on the calling thread
        }
    }
    one(0);
    for (uint32_t i : inline_ranges) one(i);
    for (auto& t : th) t.join();
    for (uint32_t i = 0; i < ns; ++i)
        if (rcs[i] < 0) return fail(rcs[i], errs[i]);
    return NFEC_OK;
}

static int run_host_batch(nfec_codec* c, const nfec_block_batch* hb, const uint16_t* locs, uint32_t lstride,
                          const uint16_t* counts, int32_t* status, bool decode)
{
    int rc = check_batch(c, hb);
    if (rc || hb->nblocks == 0) return rc;
    if (!c->stripes.empty())
        return run_striped(c, hb->nblocks, [&](nfec_codec* sc, uint32_t b0, uint32_t nb) {
            nfec_block_batch sub = *hb;
            sub.blocks = static_cast<uint8_t*>(hb->blocks) + (uint64_t)b0 * hb->block_stride;
            sub.nblocks = nb;
            sub.num_data = hb->num_data ? hb->num_data + b0 : nullptr;
            return run_host_batch(sc, &sub, locs ? locs + (uint64_t)b0 * lstride : nullptr, lstride,
                                  counts ? counts + b0 : nullptr, status ? status + b0 : nullptr, decode);
        });
    // numData is on the host here: reject what no block of k + m slots can hold before any
    // transfer is sized from it (as run_host_vectors does)
    if (hb->num_data)
        for (uint32_t b = 0; b < hb->nblocks; ++b)
            if (hb->num_data[b] == 0 || hb->num_data[b] > c->k) return fail(NFEC_EINVAL, "num_data out of range");
    DeviceGuard g(c->device);
    std::lock_guard<std::mutex> stage_lock(c->stage_mu);
    const uint64_t hbs = hb->block_stride;
    const uint64_t ss = hb->seg_stride;
    const uint64_t dbs = (uint64_t)(c->k + c->m) * ss;       // compact device pitch
    const uint64_t span = (uint64_t)(c->k + c->m - 1) * ss + c->vec;  // bytes a block op can touch
    const bool acc = (hb->flags & NFEC_ACCUMULATE) != 0;
    const bool partial_enc = !decode && !acc && !hb->num_data;
    const uint64_t up_off = 0;
    const uint64_t up_len = partial_enc ? (uint64_t)(c->k - 1) * ss + c->vec : span;
    const uint64_t dn_off = partial_enc ? (uint64_t)c->k * ss : 0;
    const uint64_t dn_len = partial_enc ? (uint64_t)(c->m - 1) * ss + c->vec
                                        : (decode ? (uint64_t)(c->k - 1) * ss + c->vec : span);
    // download pieces: parity slots one by one when slots carry padding (so the caller's
    // bytes between vec and seg_stride are never overwritten)
    std::vector<std::pair<uint64_t, uint64_t>> dn;
    if (partial_enc && ss != c->vec)
        for (uint32_t p = 0; p < c->m; ++p) dn.emplace_back((uint64_t)(c->k + p) * ss, (uint64_t)c->vec);
    else
        dn.emplace_back(dn_off, dn_len);
    const bool pinned = host_is_pinned(hb->blocks);
    uint8_t* const hbase = static_cast<uint8_t*>(hb->blocks);
    // Decode moves its bytes by zero-copy kernels (launch_slot_move): up only the slots the
    // decode reads (surviving source + the first e surviving parities; an erased source slot
    // only when accumulating), down only the repaired source slots of blocks with status > 0.
    // Per RS8(64,32) block with 16 source erasures that is 64 segments up and 16 down, against
    // 80 and 64 for the window DMA below, which stays for encode and for device setups where
    // the host memory is not mapped.
    uint8_t* const hbase_dev = pinned ? host_device_ptr(hb->blocks) : nullptr;
    const bool zc = decode && (pinned ? hbase_dev != nullptr : true) && (uint64_t)c->k + c->m <= 65536;
    // RS decode reads the source slots and only the first e surviving parities of a block (P,
    // normEncoderRS8.cpp:680-700), so a chunk's upload stops after the last parity slot any of
    // its blocks uses: [0, k + 16) instead of the whole span for RS8(64,32) with 16 source
    // erasures.  MDP decode reads every surviving vector (normEncoderMDP.cpp:346-361).
    // The download then covers [0, max numData) of the chunk, which the upload always includes
    // (slots past the upload hold another chunk's bytes and must not travel back).
    auto decode_up_len = [&](uint32_t b0, uint32_t nb, uint64_t& down) -> uint64_t {
        down = dn_len;
        if (c->kind == NFEC_MDP) return span;
        uint32_t top = 0, ndmax = 0;  // slots [0, top) are read by some block of the chunk
        std::vector<uint8_t> erased(c->k + c->m);
        for (uint32_t b = b0; b < b0 + nb; ++b) {
            const uint32_t nd = hb->num_data ? hb->num_data[b] : c->k;
            const uint32_t ec = std::min<uint32_t>(counts[b], lstride);
            const uint16_t* l = locs + (uint64_t)b * lstride;
            const uint32_t nvec = nd + c->m;
            if (nd == 0 || nd > c->k) return span;
            ndmax = std::max(ndmax, nd);
            std::fill(erased.begin(), erased.begin() + nvec, 0);
            uint32_t es = 0;
            for (uint32_t i = 0; i < ec; ++i) {
                if (l[i] >= nvec) return span;  // invalid list: the plan rejects it, stay safe
                erased[l[i]] = 1;
                es += l[i] < nd;
            }
            uint32_t used = 0, end = nd;
            for (uint32_t v = nd; v < nvec && used < es; ++v)
                if (!erased[v]) {
                    ++used;
                    end = v + 1;
                }
            if (used < es) return span;  // undecodable: nothing is read, but keep it simple
            top = std::max(top, end);
        }
        down = (uint64_t)(ndmax - 1) * ss + c->vec;
        return (uint64_t)(top - 1) * ss + c->vec;  // top >= ndmax >= 1
    };

    const uint32_t chunk = host_chunk(c, dbs, hb->nblocks);
    const uint32_t used = std::min<uint32_t>(kHostSlots, (hb->nblocks + chunk - 1) / chunk);
    const size_t meta = (size_t)chunk * (1 + lstride + 1);
    HostSlot* sl[kHostSlots] = {};
    for (uint32_t i = 0; i < used; ++i)
        if ((rc = stage_slot(c, i, (size_t)chunk * dbs, pinned ? 0 : (size_t)chunk * dbs, meta * 2 + 16,
                             (size_t)chunk * 4 + 16, sl[i])))
            return rc;
    struct Job {
        uint32_t b0 = 0, nb = 0;
        uint64_t dl = 0;  // decode: download length of the chunk's single piece
        bool busy = false;
    } jobs[kHostSlots];
    auto finish = [&](uint32_t i) -> int {
        Job& j = jobs[i];
        HostSlot& s = *sl[i];
        if (!j.busy) return NFEC_OK;
        j.busy = false;
        NFEC_HIP(hipEventSynchronize(s.done));
        if (!pinned)
            for (const auto& pc : dn)
                if (const int rc = copy2d(hbase + (uint64_t)j.b0 * hbs + pc.first, hbs, s.pin + pc.first, dbs,
                                          decode ? j.dl : pc.second, j.nb))
                    return rc;
        if (decode && status) std::memcpy(status + j.b0, s.hstat, (size_t)j.nb * 4);
        return NFEC_OK;
    };
    auto bail = [&](int code) {
        stage_drain(c);
        return code;
    };
    uint32_t idx = 0;
    for (uint32_t b0 = 0; b0 < hb->nblocks; b0 += chunk, ++idx) {
        const uint32_t i = idx % used;
        if ((rc = finish(i))) return bail(rc);
        HostSlot& s = *sl[i];
        Job& j = jobs[i];
        j.b0 = b0;
        j.nb = std::min(chunk, hb->nblocks - b0);
        uint8_t* hsrc = hbase + (uint64_t)b0 * hbs;
        uint64_t dl = dn_len;
        const uint64_t ul = decode ? decode_up_len(b0, j.nb, dl) : up_len;
        j.dl = dl;
        hipError_t ae;
        // (a pageable caller's chunk goes through the slot's pinned staging, which the zero-copy
        // kernels need device-mapped; where it is not, the window DMA below takes the chunk)
        if (zc && (pinned || s.pin_dev)) {
            if ((rc = host_decode_zc(c, hb, s, b0, j.nb, chunk, locs, lstride, counts, pinned ? hbase_dev : nullptr,
                                     ul)))
                return bail(rc);
            j.busy = true;
            continue;
        }
        if (pinned) {
            ae = hipMemcpy2DAsync(s.dev + up_off, dbs, hsrc + up_off, hbs, ul, j.nb, hipMemcpyHostToDevice, s.st);
        } else {
            if ((rc = copy2d(s.pin + up_off, dbs, hsrc + up_off, hbs, ul, j.nb))) return bail(rc);
            ae = hipMemcpyAsync(s.dev, s.pin, (size_t)(j.nb - 1) * dbs + up_off + ul, hipMemcpyHostToDevice, s.st);
        }
        uint16_t* dnd = nullptr;
        if (hb->num_data) {
            dnd = s.dmeta;
            if (ae == hipSuccess) ae = meta_up(s, dnd, hb->num_data + b0, j.nb);
        }
        nfec_block_batch db = *hb;
        db.blocks = s.dev;
        db.block_stride = dbs;
        db.nblocks = j.nb;
        db.num_data = dnd;
        if (ae != hipSuccess) return bail(hip_fail(ae, "host batch upload"));
        if (decode) {
            uint16_t* dlocs = s.dmeta + chunk;
            uint16_t* dcnt = dlocs + (size_t)chunk * lstride;
            ae = meta_up(s, dlocs, locs + (uint64_t)b0 * lstride, j.nb * lstride);
            if (ae == hipSuccess) ae = meta_up(s, dcnt, counts + b0, j.nb);
            if (ae != hipSuccess) return bail(hip_fail(ae, "host batch upload"));
            rc = split_full_runs(hb->num_data ? hb->num_data + b0 : nullptr, j.nb, c->k,
                                 [&](uint32_t o, uint32_t n, bool nd) {
                                     nfec_block_batch sb = db;
                                     sb.blocks = s.dev + o * dbs;
                                     sb.nblocks = n;
                                     sb.num_data = nd ? dnd + o : nullptr;
                                     return decode_serialized(c, &sb, dlocs + (uint64_t)o * lstride, lstride, dcnt + o, s, o);
                                 });
        } else {
            rc = split_full_runs(hb->num_data ? hb->num_data + b0 : nullptr, j.nb, c->k,
                                 [&](uint32_t o, uint32_t n, bool nd) {
                                     nfec_block_batch sb = db;
                                     sb.blocks = s.dev + o * dbs;
                                     sb.nblocks = n;
                                     sb.num_data = nd ? dnd + o : nullptr;
                                     return encode_device(c, &sb, s.st);
                                 });
        }
        if (rc) return bail(rc);
        if (pinned)
            for (size_t q = 0; q < dn.size() && ae == hipSuccess; ++q)
                ae = hipMemcpy2DAsync(hsrc + dn[q].first, hbs, s.dev + dn[q].first, dbs, decode ? dl : dn[q].second,
                                      j.nb, hipMemcpyDeviceToHost, s.st);
        else
            ae = hipMemcpyAsync(s.pin + dn_off, s.dev + dn_off, (size_t)(j.nb - 1) * dbs + (decode ? dl : dn_len),
                                hipMemcpyDeviceToHost, s.st);
        if (ae == hipSuccess && decode && status)
            ae = hipMemcpyAsync(s.hstat, s.dstat, (size_t)j.nb * 4, hipMemcpyDeviceToHost, s.st);
        if (ae == hipSuccess) ae = hipEventRecord(s.done, s.st);
        if (ae != hipSuccess) return bail(hip_fail(ae, "host batch copy"));
        j.busy = true;
    }
    for (uint32_t q = 0; q < used; ++q)
        if ((rc = finish((idx + q) % used))) return bail(rc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return bail(hip_fail(e, "host batch"));
    return NFEC_OK;
}

// ---- host segment lists (NORM's scattered segment pool) ----
// NormObject::CalculateBlockParity (src/common/normObject.cpp:2203-2229) and the receiver's
// NormSenderNode::Decode path (normObject.cpp:1548-1644) hold a block as a list of segment
// pointers from the segment pool (normSegment.cpp:14-86), not as one strided buffer.  These
// batches gather the listed segments into pinned staging (host threads), run the device
// kernels over a 3-slot H2D || compute || D2H pipeline, and scatter back only the bytes the
// reference writes: parity slots for encode, the erased source slots for decode (RS16: the
// even part of vector_size; an odd last byte is never written, normEncoderRS16.cpp:479).
namespace {

extern "C++" template <typename F>
int parallel_blocks(uint32_t nb, uint64_t bytes, F fn)
{
    const unsigned nt = (unsigned)std::min<uint64_t>(std::min<uint64_t>(host_copy_threads(), nb),
                                                      std::max<uint64_t>(1, bytes >> 22));
    if (nt <= 1) {
        fn(0u, nb);
        return NFEC_OK;
    }
    const uint32_t per = (nb + nt - 1) / nt;
    return host_parallel_for(nt, [&](unsigned t) {
        const uint32_t b0 = std::min<uint32_t>(nb, t * per), b1 = std::min<uint32_t>(nb, b0 + per);
        if (b0 < b1) fn(b0, b1);
    });
}

// the segment-list gather of blocks [b0, b0 + nb): block b's slots [0, numData_b + extra) from
// its pointer list (vecs[b * n + s]; NULL: zero) into dst + (b - b0) * dbs + s * ss, on the host
// pool.  extra: m when the parity is read too (decode, accumulate), else 0.
int gather_segments(uint8_t* dst, uint64_t dbs, uint64_t ss, void* const* vecs, uint32_t n, uint32_t b0, uint32_t nb,
                     const uint16_t* num_data, uint32_t k, uint32_t extra, uint32_t vec)
{
    return parallel_blocks(nb, (uint64_t)nb * n * vec, [&](uint32_t i0, uint32_t i1) {
        for (uint32_t i = i0; i < i1; ++i) {
            const uint32_t b = b0 + i;
            const uint32_t up = (num_data ? num_data[b] : k) + extra;
            uint8_t* d = dst + (uint64_t)i * dbs;
            for (uint32_t q = 0; q < up; ++q) {
                const void* p = vecs[(uint64_t)b * n + q];
                if (p) std::memcpy(d + q * ss, p, vec);
                else std::memset(d + q * ss, 0, vec);
            }
        }
    });
}

}  // namespace

static int run_host_vectors(nfec_codec* c, void* const* vecs, uint32_t nblocks, const uint16_t* num_data,
                            const uint16_t* locs, uint32_t lstride, const uint16_t* counts, int32_t* status,
                            uint32_t flags, bool decode)
{
    if (!c || (nblocks && !vecs)) return fail(NFEC_EINVAL, "null codec or vector list");
    if (primary(c)->host_only) return host_only_fail();
    if (decode && (!locs || !counts || lstride == 0)) return fail(NFEC_EINVAL, "bad erasure arrays");
    if (nblocks == 0) return NFEC_OK;
    if (!c->stripes.empty())
        return run_striped(c, nblocks, [&](nfec_codec* sc, uint32_t b0, uint32_t nb) {
            return run_host_vectors(sc, vecs + (uint64_t)b0 * (c->k + c->m), nb, num_data ? num_data + b0 : nullptr,
                                    locs ? locs + (uint64_t)b0 * lstride : nullptr, lstride,
                                    counts ? counts + b0 : nullptr, status ? status + b0 : nullptr, flags, decode);
        });
    const uint32_t n = c->k + c->m;
    const uint64_t ss = round_up(c->vec, 8u);
    const uint64_t dbs = (uint64_t)n * ss;
    const bool acc = (flags & NFEC_ACCUMULATE) != 0;
    const size_t out_bytes = c->sym == 2 ? (c->vec & ~1u) : c->vec;
    // validate the lists (the reference dereferences every source vector and, for encode,
    // every parity vector; decode never touches missing parity, normEncoderRS8.cpp:689-711)
    for (uint32_t b = 0; b < nblocks; ++b) {
        const uint32_t nd = num_data ? num_data[b] : c->k;
        if (nd == 0 || nd > c->k) return fail(NFEC_EINVAL, "num_data out of range");
        const uint32_t need = decode ? nd : nd + c->m;
        for (uint32_t s = 0; s < need; ++s)
            if (!vecs[(uint64_t)b * n + s]) return fail(NFEC_EINVAL, "null source/parity vector");
    }
    DeviceGuard g(c->device);
    std::lock_guard<std::mutex> stage_lock(c->stage_mu);
    const uint32_t chunk = host_chunk(c, dbs, nblocks);
    const uint32_t used = std::min<uint32_t>(kHostSlots, (nblocks + chunk - 1) / chunk);
    const size_t meta = (size_t)chunk * (1 + lstride + 1);
    HostSlot* sl[kHostSlots] = {};
    int rc;
    for (uint32_t i = 0; i < used; ++i)
        if ((rc = stage_slot(c, i, (size_t)chunk * dbs, (size_t)chunk * dbs, meta * 2 + 16, (size_t)chunk * 4 + 16,
                             sl[i])))
            return rc;
    struct Job {
        uint32_t b0 = 0, nb = 0;
        uint64_t dl = 0;  // decode: download length of the chunk's single piece
        bool busy = false;
    } jobs[kHostSlots];
    auto gather = [&](HostSlot& s, const Job& j) {
        // encode without accumulate reads the source only; everything else reads the whole
        // listed block (absent parity is zero, as MDP's decoder treats it)
        return gather_segments(s.pin, dbs, ss, vecs, n, j.b0, j.nb, num_data, c->k, (!decode && !acc) ? 0u : c->m,
                               c->vec);
    };
    auto scatter = [&](HostSlot& s, const Job& j) {
        return parallel_blocks(j.nb, (uint64_t)j.nb * (uint64_t)c->m * c->vec, [&](uint32_t i0, uint32_t i1) {
            for (uint32_t i = i0; i < i1; ++i) {
                const uint32_t b = j.b0 + i;
                const uint32_t nd = num_data ? num_data[b] : c->k;
                const uint8_t* src = s.pin + (uint64_t)i * dbs;
                if (!decode) {
                    for (uint32_t p = 0; p < c->m; ++p)
                        std::memcpy(vecs[(uint64_t)b * n + nd + p], src + (nd + p) * ss, out_bytes);
                } else if (s.hstat[i] > 0) {
                    const uint16_t* l = locs + (uint64_t)b * lstride;
                    for (uint32_t e = 0; e < counts[b] && e < lstride; ++e) {
                        if (l[e] >= nd) break;  // only source erasures are filled (normEncoderRS8.cpp:732)
                        std::memcpy(vecs[(uint64_t)b * n + l[e]], src + l[e] * ss, out_bytes);
                    }
                }
            }
        });
    };
    auto finish = [&](uint32_t i) -> int {
        Job& j = jobs[i];
        if (!j.busy) return NFEC_OK;
        j.busy = false;
        NFEC_HIP(hipEventSynchronize(sl[i]->done));
        if (const int rc = scatter(*sl[i], j)) return rc;
        if (decode && status) std::memcpy(status + j.b0, sl[i]->hstat, (size_t)j.nb * 4);
        return NFEC_OK;
    };
    auto bail = [&](int code) {
        stage_drain(c);
        return code;
    };
    uint32_t idx = 0;
    for (uint32_t b0 = 0; b0 < nblocks; b0 += chunk, ++idx) {
        const uint32_t i = idx % used;
        if ((rc = finish(i))) return bail(rc);
        HostSlot& s = *sl[i];
        Job& j = jobs[i];
        j.b0 = b0;
        j.nb = std::min(chunk, nblocks - b0);
        if ((rc = gather(s, j))) return bail(rc);
        // decode: the staged slots the decode reads go up by the zero-copy gather kernel (the
        // erased source and unused parity stay on the host), the repaired ones come down by
        // the scatter kernel (launch_slot_move, as in run_host_batch)
        const bool zcv = decode && s.pin_dev && (uint64_t)n <= 65536;
        hipError_t ae = zcv ? hipSuccess : hipMemcpyAsync(s.dev, s.pin, (size_t)j.nb * dbs, hipMemcpyHostToDevice, s.st);
        uint16_t* dnd = nullptr;
        if (num_data && ae == hipSuccess) {
            dnd = s.dmeta;
            ae = meta_up(s, dnd, num_data + b0, j.nb);
        }
        if (ae != hipSuccess) return bail(hip_fail(ae, "vector batch upload"));
        nfec_block_batch db;
        std::memset(&db, 0, sizeof(db));
        db.blocks = s.dev;
        db.block_stride = dbs;
        db.seg_stride = (uint32_t)ss;
        db.nblocks = j.nb;
        db.num_data = dnd;
        db.flags = flags;
        if (decode) {
            uint16_t* dl = s.dmeta + chunk;
            uint16_t* dc = dl + (size_t)chunk * lstride;
            ae = meta_up(s, dl, locs + (uint64_t)b0 * lstride, j.nb * lstride);
            if (ae == hipSuccess) ae = meta_up(s, dc, counts + b0, j.nb);
            if (ae != hipSuccess) return bail(hip_fail(ae, "vector batch upload"));
            SlotMoveArgs mv;
            if (zcv) {
                mv.src = s.pin_dev;
                mv.src_block_stride = dbs;
                mv.src_seg_stride = (uint32_t)ss;
                mv.dst = s.dev;
                mv.dst_block_stride = dbs;
                mv.dst_seg_stride = (uint32_t)ss;
                mv.nblocks = j.nb;
                mv.k = c->k;
                mv.m = c->m;
                mv.bytes = c->vec;
                mv.num_data = dnd;
                mv.locs = dl;
                mv.lstride = lstride;
                mv.counts = dc;
                mv.mode = c->kind == NFEC_MDP ? SLOTS_ALL_IN : SLOTS_RS_IN;
                mv.accumulate = acc ? 1u : 0u;
                if ((rc = launch_slot_move(mv, s.st))) return bail(rc);
            }
            rc = split_full_runs(num_data ? num_data + b0 : nullptr, j.nb, c->k, [&](uint32_t o, uint32_t n, bool nd) {
                nfec_block_batch sb = db;
                sb.blocks = s.dev + o * dbs;
                sb.nblocks = n;
                sb.num_data = nd ? dnd + o : nullptr;
                return decode_serialized(c, &sb, dl + (uint64_t)o * lstride, lstride, dc + o, s, o);
            });
            if (!rc && zcv) {
                SlotMoveArgs out = mv;
                out.src = s.dev;
                out.dst = s.pin_dev;
                out.bytes = (uint32_t)out_bytes;
                out.status = s.dstat;
                out.mode = SLOTS_OUT;
                rc = launch_slot_move(out, s.st);
            }
            if (!rc) {
                ae = hipMemcpyAsync(s.hstat, s.dstat, (size_t)j.nb * 4, hipMemcpyDeviceToHost, s.st);
                if (ae != hipSuccess) return bail(hip_fail(ae, "vector batch status"));
            }
        } else {
            rc = split_full_runs(num_data ? num_data + b0 : nullptr, j.nb, c->k, [&](uint32_t o, uint32_t n, bool nd) {
                nfec_block_batch sb = db;
                sb.blocks = s.dev + o * dbs;
                sb.nblocks = n;
                sb.num_data = nd ? dnd + o : nullptr;
                return encode_device(c, &sb, s.st);
            });
        }
        if (rc) return bail(rc);
        // unshortened encode: only the parity region of each block comes back
        if (zcv)
            ae = hipSuccess;
        else if (!decode && !num_data)
            ae = hipMemcpy2DAsync(s.pin + (uint64_t)c->k * ss, dbs, s.dev + (uint64_t)c->k * ss, dbs, (uint64_t)c->m * ss,
                                  j.nb, hipMemcpyDeviceToHost, s.st);
        else
            ae = hipMemcpyAsync(s.pin, s.dev, (size_t)j.nb * dbs, hipMemcpyDeviceToHost, s.st);
        if (ae == hipSuccess) ae = hipEventRecord(s.done, s.st);
        if (ae != hipSuccess) return bail(hip_fail(ae, "vector batch download"));
        j.busy = true;
    }
    for (uint32_t q = 0; q < used; ++q)
        if ((rc = finish((idx + q) % used))) return bail(rc);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return bail(hip_fail(e, "vector batch"));
    return NFEC_OK;
}

int nfec_encode_host_vectors(nfec_codec* codec, void* const* vectors, uint32_t nblocks, const uint16_t* num_data,
                             uint32_t flags)
{
    return run_host_vectors(codec, vectors, nblocks, num_data, nullptr, 0, nullptr, nullptr, flags, false);
}

int nfec_decode_host_vectors(nfec_codec* codec, void* const* vectors, uint32_t nblocks, const uint16_t* num_data,
                             const uint16_t* erasure_locs, uint32_t erasure_stride, const uint16_t* erasure_counts,
                             int32_t* status, uint32_t flags)
{
    return run_host_vectors(codec, vectors, nblocks, num_data, erasure_locs, erasure_stride, erasure_counts, status,
                            flags, true);
}

int nfec_encode_host(nfec_codec* codec, const nfec_block_batch* host_batch)
{
    return run_host_batch(codec, host_batch, nullptr, 0, nullptr, nullptr, false);
}

int nfec_decode_host(nfec_codec* codec, const nfec_block_batch* host_batch, const uint16_t* erasure_locs,
                     uint32_t erasure_stride, const uint16_t* erasure_counts, int32_t* status)
{
    if (!erasure_locs || !erasure_counts || erasure_stride == 0) return fail(NFEC_EINVAL, "bad erasure arrays");
    return run_host_batch(codec, host_batch, erasure_locs, erasure_stride, erasure_counts, status, true);
}

// ---- asynchronous segment-list batches (receiver cross-block batching) ----
// The receiver's decode site (NormObject::HandleObjectMessage -> NormSenderNode::Decode,
// normObject.cpp:1548-1644, normNode.h:484-487) repairs one block per call on the protocol
// thread.  These calls queue many blocks (from one remote sender's decoder) and return at
// once; the protocol thread keeps receiving and collects completions with nfec_request_test /
// nfec_request_wait.  The pointer table, numData, erasure lists and counts are copied at
// submission; the segment buffers and status array must stay valid until completion.
namespace {

int submit_vectors(nfec_codec* c, void* const* vecs, uint32_t nblocks, const uint16_t* num_data, const uint16_t* locs,
                   uint32_t lstride, const uint16_t* counts, int32_t* status, uint32_t flags, bool decode,
                   nfec_request** out)
{
    if (!out) return fail(NFEC_EINVAL, "null request pointer");
    *out = nullptr;
    if (!c || (nblocks && !vecs)) return fail(NFEC_EINVAL, "null codec or vector list");
    if (primary(c)->host_only) return host_only_fail();
    if (decode && (!locs || !counts || lstride == 0)) return fail(NFEC_EINVAL, "bad erasure arrays");
    const uint64_t n = (uint64_t)c->k + c->m;
    auto tab = std::make_shared<std::vector<void*>>(vecs, vecs + n * nblocks);
    auto nd = std::make_shared<std::vector<uint16_t>>();
    if (num_data) nd->assign(num_data, num_data + nblocks);
    auto el = std::make_shared<std::vector<uint16_t>>();
    auto ec = std::make_shared<std::vector<uint16_t>>();
    if (decode) {
        el->assign(locs, locs + (uint64_t)lstride * nblocks);
        ec->assign(counts, counts + nblocks);
    }
    std::unique_ptr<nfec_request> r(new nfec_request);
    r->run = [=]() {
        return run_host_vectors(c, tab->data(), nblocks, num_data ? nd->data() : nullptr,
                                decode ? el->data() : nullptr, lstride, decode ? ec->data() : nullptr, status,
                                flags, decode);
    };
    c->async.submit(r.get());
    *out = r.release();
    return NFEC_OK;
}

}  // namespace

int nfec_encode_host_vectors_async(nfec_codec* codec, void* const* vectors, uint32_t nblocks, const uint16_t* num_data,
                                   uint32_t flags, nfec_request** request)
{
    return submit_vectors(codec, vectors, nblocks, num_data, nullptr, 0, nullptr, nullptr, flags, false, request);
}

int nfec_decode_host_vectors_async(nfec_codec* codec, void* const* vectors, uint32_t nblocks,
                                   const uint16_t* num_data, const uint16_t* erasure_locs, uint32_t erasure_stride,
                                   const uint16_t* erasure_counts, int32_t* status, uint32_t flags,
                                   nfec_request** request)
{
    return submit_vectors(codec, vectors, nblocks, num_data, erasure_locs, erasure_stride, erasure_counts, status,
                          flags, true, request);
}

int nfec_request_test(nfec_request* r)
{
    if (!r) return fail(NFEC_EINVAL, "null request");
    std::lock_guard<std::mutex> lk(r->mu);
    return r->done ? 1 : 0;
}

int nfec_request_wait(nfec_request* r)
{
    if (!r) return fail(NFEC_EINVAL, "null request");
    int rc;
    std::string err;
    {
        std::unique_lock<std::mutex> lk(r->mu);
        r->cv.wait(lk, [&] { return r->done; });
        rc = r->rc;
        err.swap(r->err);
    }
    delete r;
    return rc < 0 ? fail(rc, err) : rc;
}

// ---- synthetic workload utilities ----
int nfec_util_fill(const nfec_block_batch* b, uint32_t num_data, uint32_t vector_size, uint64_t seed,
                   uint64_t first_block, void* stream)
{
    if (!b || !b->blocks) return fail(NFEC_EINVAL, "null batch");
    return launch_fill(static_cast<uint8_t*>(b->blocks), b->block_stride, b->seg_stride, b->nblocks, b->num_data,
                       num_data, vector_size, seed, first_block, static_cast<hipStream_t>(stream));
}

int nfec_util_erasures(uint16_t* locs, uint32_t stride, uint16_t* counts, uint32_t nblocks, uint32_t range,
                       uint32_t count, uint64_t seed, uint64_t first_block, void* stream)
{
    if (!locs || !counts || stride == 0) return fail(NFEC_EINVAL, "bad erasure arrays");
    return launch_erasures(locs, stride, counts, nblocks, range, count, seed, first_block,
                           static_cast<hipStream_t>(stream));
}

int nfec_util_zero_slots(const nfec_block_batch* b, const uint16_t* locs, uint32_t stride, const uint16_t* counts,
                         uint32_t vector_size, void* stream)
{
    if (!b || !b->blocks || !locs || !counts) return fail(NFEC_EINVAL, "null argument");
    return launch_zero_slots(static_cast<uint8_t*>(b->blocks), b->block_stride, b->seg_stride, b->nblocks, locs,
                             stride, counts, vector_size, static_cast<hipStream_t>(stream));
}

int nfec_host_threads(uint32_t* pool, uint32_t* usable_cores, uint32_t* visible_cores)
{
    if (pool) *pool = host_pool_workers();
    if (usable_cores) *usable_cores = host_usable_cores();
    if (visible_cores) *visible_cores = host_visible_cores();
    return NFEC_OK;
}

int nfec_util_pool_check(uint32_t pieces, int mode)
{
    if (mode < 0 || mode > 2 || (mode && pieces < 2)) return fail(NFEC_EINVAL, "bad argument");
    std::atomic<uint32_t> ran{0};
    const int rc = host_parallel_for(pieces, [&](unsigned i) {
        if (mode == 1 && i == 1) throw std::bad_alloc();
        if (mode == 2 && i == 1) throw std::runtime_error("pool check");
        ran.fetch_add(1);
    });
    return rc ? rc : (int)ran.load();
}

int nfec_util_gather_probe(void* const* vectors, uint32_t nblocks, uint32_t slots, uint32_t vector_size,
                           uint32_t nstripes, uint32_t reps, double* seconds, uint32_t* max_active)
{
    if (!vectors || !seconds || nblocks == 0 || slots == 0 || vector_size == 0 || nstripes == 0 || nstripes > 64 ||
        reps == 0)
        return fail(NFEC_EINVAL, "bad argument");
    const uint64_t ss = round_up(vector_size, 8u), dbs = (uint64_t)slots * ss;
    const uint32_t chunk = (uint32_t)std::max<uint64_t>(1, (128ull << 20) / dbs);  // the pipelines' 128 MiB chunks
    std::vector<std::unique_ptr<uint8_t, void (*)(void*)>> stage;
    for (uint32_t i = 0; i < nstripes; ++i) {
        const uint64_t nb = (uint64_t)nblocks * (i + 1) / nstripes - (uint64_t)nblocks * i / nstripes;
        void* p = nullptr;
        const size_t bytes = (size_t)std::max<uint64_t>(1, std::min<uint64_t>(nb, chunk)) * dbs;
        if (posix_memalign(&p, 4096, bytes)) return fail(NFEC_ENOMEM, "probe staging");
        std::memset(p, 0, bytes);  // touched before timing
        stage.emplace_back(static_cast<uint8_t*>(p), std::free);
    }
    auto stripe = [&](uint32_t i) {
        const uint32_t lo = (uint32_t)((uint64_t)nblocks * i / nstripes), hi = (uint32_t)((uint64_t)nblocks * (i + 1) / nstripes);
        for (uint32_t b0 = lo; b0 < hi; b0 += chunk)
            (void)gather_segments(stage[i].get(), dbs, ss, vectors, slots, b0, std::min(chunk, hi - b0), nullptr, slots,
                                  0, vector_size);
    };
    auto pass = [&] {
        std::vector<std::thread> th;
        for (uint32_t i = 1; i < nstripes; ++i) th.emplace_back(stripe, i);
        stripe(0);
        for (auto& t : th) t.join();
    };
    pass();  // untimed: first touches of the pool, the table and the staging
    if (max_active) host_pool_max_active(true);
    const auto t0 = std::chrono::steady_clock::now();
    for (uint32_t r = 0; r < reps; ++r) pass();
    *seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() / reps;
    if (max_active) *max_active = host_pool_max_active(false);
    return NFEC_OK;
}

int nfec_util_stream_copy(void* dst, const void* src, uint64_t bytes, void* stream)
{
    if ((!dst || !src) && bytes) return fail(NFEC_EINVAL, "null argument");
    return launch_stream_copy(dst, src, bytes, static_cast<hipStream_t>(stream));
}

}  // extern "C"
