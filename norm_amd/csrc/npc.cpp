// npc.cpp -- the reference's offline file precoder (src/common/normPrecode.cpp, "npc") with
// the FEC and checksum work on the GPU.
//
// File format (byte-identical to the reference's output on the same input and parameters):
//   * input segment 0 is a meta segment: the file size (8 bytes, big-endian) and the input
//     file's base name (normPrecode.cpp:650-678); then the file in segment_size - 4 byte
//     pieces, the last one zero-padded (:718-740);
//   * FEC blocks of numData input segments (the last block shorter), each followed by its
//     numParity parity segments, RS8 when numData + numParity <= 256, RS16 above (:624-628);
//   * every segment ends in a big-endian CRC-32 of its first segment_size - 4 bytes (:780-783);
//   * segments are written in interleaved order (ComputeInterleaverOffset, :465-556).
// Decode reverses this: a CRC mismatch is an erasure, the erased vectors are zeroed and the
// block goes through the RS decoder (:1039-1050, :1077-1089, :1126-1128).
//
// The reference encoder passes outputSegmentId % numData as the Encode() segment id
// (:746), and outputSegmentId counts the parity segments of earlier blocks too, so block b's
// source segment i is coded as generator column (b*numParity + i) mod numData.  Its decoder
// uses column i (:1128).  Both are reproduced here, so .npc files and decoded output match
// the reference byte for byte -- including the reference's wrong repairs in blocks whose
// rotation is not zero (npc).
//
// GPU work per chunk of blocks: H2D, nfec_encode (or CRC check -> erasure lists -> zero ->
// nfec_decode), CRC-32 of every segment, D2H.  Host threads gather and scatter segments
// between the memory-mapped files and pinned staging; two staging slots overlap one chunk's
// host work with the next chunk's GPU work.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "nfec_internal.hpp"

using namespace nfec;

namespace {

constexpr uint32_t kSegMin = 12;    // reference SEGMENT_MIN is 8, but below 12 its meta segment
constexpr uint32_t kSegMax = 8192;  // overflows (strncpy of segment_size - 12 bytes, :678)
constexpr uint64_t kBlockMax = 65536;

uint32_t round8(uint32_t v) { return (v + 7u) & ~7u; }

void put_be32(uint8_t* p, uint32_t v)
{
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

// InitInterleaver (normPrecode.cpp:450-462)
void init_interleaver(nfec_npc_layout* l)
{
    const int64_t n = (int64_t)l->num_segments;
    int64_t w = (int64_t)std::sqrt((double)n);
    int64_t h = n / w;
    if (n % h) h++;
    const int64_t imax = (int64_t)l->i_max;
    if (imax > 0 && (w > imax || h > imax)) h = w = imax;
    l->il_width = (uint64_t)w;
    l->il_height = (uint64_t)h;
    l->il_size = (uint64_t)(w * h);
}

// ComputeInterleaverOffset / segment_size (normPrecode.cpp:465-556): the file slot of FEC-order
// segment `seg`.  Signed 64-bit like ProtoFile::Offset.  Returns -1 where the reference would
// divide by zero or leave the file (its ASSERTs are compiled out in release builds).
int64_t il_position(const nfec_npc_layout* l, int64_t seg)
{
    const int64_t n = (int64_t)l->num_segments;
    const int64_t size = (int64_t)l->il_size;
    int64_t w = (int64_t)l->il_width, h = (int64_t)l->il_height;
    int64_t blk = 0;
    if (l->i_max > 0) {
        blk = seg / size;
        seg = seg % size;
    }
    const int64_t last = n - 1;
    if (blk == last / size && n % size) {
        const int64_t lbs = n % size;
        w = (int64_t)std::sqrt((double)lbs);
        h = lbs / w;
        if (lbs % h) h++;
    }
    int64_t col = seg / h, row = seg % h;
    int64_t id = row * w + col;
    if (blk) id += blk * size;
    if (id >= n) {
        int64_t lastId = n - 1;
        if (blk) {
            id = id % size;
            lastId = lastId % size;
        }
        const int64_t maxRow = lastId / w, maxCol = lastId % w;
        const int64_t emptyRows = h - maxRow - 1;
        int64_t delta = 1 + emptyRows * col;
        if (col > maxCol) {
            delta += row - maxRow;
            delta += col - maxCol - 1;
        } else {
            delta += row - maxRow - 1;
        }
        int64_t lastCol = lastId / h, lastRow = lastId % h;
        lastRow += delta;
        if (lastCol == maxCol && lastRow > maxRow) {
            lastCol++;
            lastRow -= maxRow + 1;
        }
        if (maxRow == 0) return -1;
        col = lastCol + lastRow / maxRow;
        row = lastRow % maxRow;
        id = row * w + col;
        if (blk) id += blk * size;
    }
    return (id >= 0 && id < n) ? id : -1;
}

// Auto block sizing and parameter checks (NormPrecodeApp::OnStartup, normPrecode.cpp:383-434).
int resolve(const nfec_npc_params* p, uint64_t file_size, int encode, uint32_t* k, uint32_t* m)
{
    uint32_t nd = p->num_data, np = p->num_parity;
    if (p->parity_fraction >= 0.0) {
        uint32_t bs;
        if (encode) {
            bs = (uint32_t)(file_size / (p->segment_size - 4));
            if (file_size % (p->segment_size - 4)) bs += 1;
            bs += 1;  // meta segment
        } else {
            const uint64_t ns = file_size / p->segment_size;
            bs = (uint32_t)(((double)ns / (1.0 + p->parity_fraction)) + 0.5);
        }
        if (bs > p->b_max) bs = (uint32_t)p->b_max;
        uint32_t par = (uint32_t)((p->parity_fraction * bs) + 0.5);
        if ((uint64_t)bs + par > kBlockMax) {
            const double scale = (double)kBlockMax / ((double)bs + (double)par);
            bs = (uint32_t)(scale * bs);
            par = (uint32_t)(scale * par);
        }
        nd = bs;
        np = par;
    }
    if ((uint64_t)nd + np > kBlockMax) return fail(NFEC_ERANGE, "npc: numData/numParity total exceeds max block size");
    if (nd == 0) return fail(NFEC_EINVAL, "npc: numData is 0");
    if (np == 0) return fail(NFEC_EINVAL, "npc: numParity 0 is not supported (the reference indexes an empty parity list)");
    *k = nd;
    *m = np;
    return NFEC_OK;
}

struct Threads {
    // host copy threads of a file pass (NFEC_NPC_THREADS, default min(16, cores)), shared
    // evenly by its device workers
    static unsigned total()
    {
        static const unsigned nt = [] {
            const char* e = std::getenv("NFEC_NPC_THREADS");
            const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
            return e ? std::max(1, std::atoi(e)) : std::min(16u, hw);
        }();
        return nt;
    }
    // run f(lo, hi) over [0, n) split across up to nt host threads
    template <typename F>
    static void run(uint64_t n, unsigned nt, F f)
    {
        const unsigned t = (unsigned)std::min<uint64_t>(std::max(1u, nt), std::max<uint64_t>(1, n / 4));
        if (t <= 1) {
            f(0, n);
            return;
        }
        std::vector<std::thread> pool;
        for (unsigned i = 0; i < t; ++i) {
            const uint64_t lo = n * i / t, hi = n * (i + 1) / t;
            try {
                pool.emplace_back([=] { f(lo, hi); });
            } catch (...) {
                f(lo, hi);  // no thread to be had: this range on the calling thread
            }
        }
        for (auto& th : pool) th.join();
    }
};

struct MappedFile {
    int fd = -1;
    uint8_t* p = nullptr;
    uint64_t size = 0;
    ~MappedFile()
    {
        if (p && size) munmap(p, size);
        if (fd >= 0) close(fd);
    }
    int open_read(const char* path)
    {
        fd = ::open(path, O_RDONLY);
        if (fd < 0) return fail(NFEC_EINVAL, std::string("npc: cannot open input file ") + path);
        struct stat st;
        if (fstat(fd, &st)) return fail(NFEC_EINVAL, "npc: stat failed");
        size = (uint64_t)st.st_size;
        if (size) {
            void* m = mmap(nullptr, size, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
            if (m == MAP_FAILED) return fail(NFEC_ENOMEM, "npc: mmap of input failed");
            p = static_cast<uint8_t*>(m);
        }
        return NFEC_OK;
    }
    int open_write(const char* path, uint64_t bytes)
    {
        fd = ::open(path, O_RDWR | O_CREAT | O_TRUNC, 0644);
        if (fd < 0) return fail(NFEC_EINVAL, std::string("npc: cannot open output file ") + path);
        if (ftruncate(fd, (off_t)bytes)) return fail(NFEC_ENOMEM, "npc: cannot size output file");
        size = bytes;
        if (size) {
            // populated up front: one kernel pass instead of a page fault per 4 KiB from the copy threads
            void* m = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, fd, 0);
            if (m == MAP_FAILED) return fail(NFEC_ENOMEM, "npc: mmap of output failed");
            p = static_cast<uint8_t*>(m);
        }
        return NFEC_OK;
    }
};

// Device + pinned staging for chunks of blocks, two slots, one stream (the codec's decode
// workspace is shared, so chunks run in order on the GPU).
struct Stage {
    int device = 0;
    hipStream_t st = nullptr;
    uint8_t* dblk = nullptr;  // [cb][k+m][stride]
    uint8_t* hblk[2] = {nullptr, nullptr};
    uint32_t* dcrc = nullptr;
    uint32_t* hcrc[2] = {nullptr, nullptr};
    uint8_t* dbad = nullptr;
    uint16_t* dnd = nullptr;
    uint16_t* hnd[2] = {nullptr, nullptr};
    uint16_t* dlocs = nullptr;
    uint16_t* dcounts = nullptr;
    uint16_t* hcounts[2] = {nullptr, nullptr};
    int32_t* dstatus = nullptr;
    hipEvent_t done[2] = {nullptr, nullptr};
    nfec_codec* codec = nullptr;

    ~Stage()
    {
        if (st) (void)hipStreamSynchronize(st);
        for (int i = 0; i < 2; ++i) {
            if (hblk[i]) (void)hipHostFree(hblk[i]);
            if (hcrc[i]) (void)hipHostFree(hcrc[i]);
            if (hnd[i]) (void)hipHostFree(hnd[i]);
            if (hcounts[i]) (void)hipHostFree(hcounts[i]);
            if (done[i]) (void)hipEventDestroy(done[i]);
        }
        for (void* p : {(void*)dblk, (void*)dcrc, (void*)dbad, (void*)dnd, (void*)dlocs, (void*)dcounts,
                        (void*)dstatus})
            if (p) (void)hipFree(p);
        if (codec) nfec_codec_destroy(codec);
        if (st) (void)hipStreamDestroy(st);
    }

    int init(int dev, const nfec_npc_layout& l, uint32_t stride, uint32_t cb)
    {
        device = dev;
        const uint32_t n = l.num_data + l.num_parity;
        const uint64_t bstride = (uint64_t)n * stride;
        int rc = nfec_codec_create(dev, l.kind, l.num_data, l.num_parity, l.segment_size - 4, &codec);
        if (rc) return rc;
        NFEC_HIP(hipSetDevice(dev));
        NFEC_HIP(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
        NFEC_HIP(hipMalloc(&dblk, bstride * cb));
        NFEC_HIP(hipMalloc(&dcrc, (size_t)cb * n * 4));
        NFEC_HIP(hipMalloc(&dbad, (size_t)cb * n));
        NFEC_HIP(hipMalloc(&dnd, (size_t)cb * 2));
        NFEC_HIP(hipMalloc(&dlocs, (size_t)cb * l.num_parity * 2));
        NFEC_HIP(hipMalloc(&dcounts, (size_t)cb * 2));
        NFEC_HIP(hipMalloc(&dstatus, (size_t)cb * 4));
        for (int i = 0; i < 2; ++i) {
            NFEC_HIP(hipHostMalloc(&hblk[i], bstride * cb, hipHostMallocDefault));
            NFEC_HIP(hipHostMalloc(&hcrc[i], (size_t)cb * n * 4, hipHostMallocDefault));
            NFEC_HIP(hipHostMalloc(&hnd[i], (size_t)cb * 2, hipHostMallocDefault));
            NFEC_HIP(hipHostMalloc(&hcounts[i], (size_t)cb * 2, hipHostMallocDefault));
            NFEC_HIP(hipEventCreateWithFlags(&done[i], hipEventDisableTiming));
        }
        return NFEC_OK;
    }
};

uint32_t chunk_blocks(uint64_t block_bytes, uint64_t nblocks)
{
    static const uint64_t budget = [] {
        const char* e = std::getenv("NFEC_NPC_CHUNK_MB");
        const long mb = e ? std::atol(e) : 256L;
        return (uint64_t)std::max(1L, mb) << 20;
    }();
    const uint64_t cb = std::max<uint64_t>(1, budget / std::max<uint64_t>(block_bytes, 1));
    return (uint32_t)std::min<uint64_t>({cb, nblocks, (uint64_t)1 << 20});
}

// NFEC_NPC_PROFILE=1: per-phase wall times of a file pass on stderr
struct Phases {
    bool on = [] {
        const char* e = std::getenv("NFEC_NPC_PROFILE");
        return e && *e && *e != '0';
    }();
    double t[6] = {0, 0, 0, 0, 0, 0};
    std::chrono::steady_clock::time_point last = std::chrono::steady_clock::now();
    void mark(int i)
    {
        const auto now = std::chrono::steady_clock::now();
        t[i] += std::chrono::duration<double>(now - last).count();
        last = now;
    }
    void report(const char* what) const
    {
        if (on)
            std::fprintf(stderr,
                         "npc %s: map input %.3f s, positions %.3f s, staging+output %.3f s, host in %.3f s, "
                         "gpu enqueue %.3f s, host out %.3f s\n",
                         what, t[4], t[5], t[0], t[1], t[2], t[3]);
    }
};

std::string base_name(const char* path)
{
    const char* s = std::strrchr(path, '/');
    return s ? s + 1 : path;
}

int check_devices(const int32_t* devices, int32_t n)
{
    if (!devices || n < 1) return fail(NFEC_EINVAL, "npc: empty device list");
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess) {
        (void)hipGetLastError();
        return fail(NFEC_EDEVICE, "npc: no HIP device");
    }
    for (int32_t i = 0; i < n; ++i)
        if (devices[i] < 0 || devices[i] >= count) return fail(NFEC_EINVAL, "npc: device index out of range");
    return NFEC_OK;
}

// the file pass over ndev devices: device i takes the contiguous block range
// [nblocks * i / ndev, nblocks * (i + 1) / ndev) through its own staging pipeline and codec, on
// its own host thread (one device: the calling thread, whose current device is restored).
// Returns the first failing worker's code in device-list order.
template <typename F>
int run_devices(const int32_t* devices, uint32_t ndev, uint64_t nblocks, F worker)
{
    if (ndev == 1) {
        int prev = -1;
        (void)hipGetDevice(&prev);
        const int rc = worker(0u, devices[0], (uint64_t)0, nblocks);
        if (prev >= 0) (void)hipSetDevice(prev);
        return rc;
    }
    // each worker's error message is thread-local: keep it and set it again on the calling thread
    // for the first failing worker (as nfec_api.cpp's run_striped does)
    std::vector<int> rcs(ndev, NFEC_OK);
    std::vector<std::string> errs(ndev);
    auto one = [&](uint32_t i) {
        rcs[i] = worker(i, devices[i], nblocks * i / ndev, nblocks * (i + 1) / ndev);
        if (rcs[i] < 0) errs[i] = last_error_cstr();
    };
    std::vector<std::thread> th;
    std::vector<uint32_t> inline_ranges;
    for (uint32_t i = 0; i < ndev; ++i) {
        try {
            th.emplace_back(one, i);
        } catch (...) {
            inline_ranges.push_back(i);  // no thread to be had: that range on the calling thread
        }
    }
    for (uint32_t i : inline_ranges) one(i);
    for (auto& t : th) t.join();
    for (uint32_t i = 0; i < ndev; ++i)
        if (rcs[i]) return rcs[i] < 0 ? fail(rcs[i], errs[i]) : rcs[i];
    return NFEC_OK;
}

}  // namespace

extern "C" {

void nfec_npc_default_params(nfec_npc_params* p)
{
    if (!p) return;
    // NormPrecodeApp::NormPrecodeApp (normPrecode.cpp:111-115)
    p->segment_size = 1024;
    p->num_data = 196;
    p->num_parity = 4;
    p->parity_fraction = 100.0;
    p->b_max = 65536;
    p->i_max = 1000;
}

int nfec_npc_layout_for(const nfec_npc_params* p, uint64_t file_size, int encode, nfec_npc_layout* out)
{
    if (!p || !out) return fail(NFEC_EINVAL, "null argument");
    if (p->segment_size < kSegMin || p->segment_size > kSegMax)
        return fail(NFEC_EINVAL, "npc: segment size out of range (12..8192)");
    uint32_t k = 0, m = 0;
    int rc = resolve(p, file_size, encode, &k, &m);
    if (rc) return rc;
    nfec_npc_layout l{};
    l.num_data = k;
    l.num_parity = m;
    l.segment_size = p->segment_size;
    l.i_max = p->i_max;
    l.kind = (k + m > 256) ? NFEC_RS16 : NFEC_RS8;
    const uint32_t ds = p->segment_size - 4;
    if (encode) {
        // NormPrecodeApp::Encode (normPrecode.cpp:611-637)
        uint64_t nin = 1 + file_size / ds;
        uint32_t last_seg = (uint32_t)(file_size % ds);
        if (last_seg) nin++;
        else last_seg = ds;
        uint64_t nb = nin / k;
        uint32_t lbs = (uint32_t)(nin % k);
        if (lbs) nb++;
        else lbs = k;
        l.num_blocks = nb;
        l.last_block_data = lbs;
        l.last_segment_bytes = last_seg;
        l.input_segments = nin;
        l.num_segments = (nb - 1) * (uint64_t)(k + m) + lbs + m;
    } else {
        // NormPrecodeApp::Decode (normPrecode.cpp:886-906)
        if (file_size % p->segment_size) return fail(NFEC_EINVAL, "npc: input file size not integral number of segments");
        const uint64_t ns = file_size / p->segment_size;
        uint64_t nb = ns / (k + m);
        uint32_t lbs = (uint32_t)(ns % (k + m));
        if (lbs) {
            if (lbs <= m) return fail(NFEC_EINVAL, "npc: last FEC block holds no source segment");
            lbs -= m;
            nb++;
        } else {
            lbs = k;
        }
        if (nb == 0) return fail(NFEC_EINVAL, "npc: empty input");
        l.num_blocks = nb;
        l.last_block_data = lbs;
        l.num_segments = ns;
        l.input_segments = (nb - 1) * (uint64_t)k + lbs;
    }
    init_interleaver(&l);
    *out = l;
    return NFEC_OK;
}

int nfec_npc_positions(const nfec_npc_layout* l, uint64_t first, uint64_t count, uint64_t* pos)
{
    if (!l || (count && !pos)) return fail(NFEC_EINVAL, "null argument");
    if (first + count > l->num_segments || l->il_size == 0) return fail(NFEC_EINVAL, "npc: segment range");
    for (uint64_t i = 0; i < count; ++i) {
        const int64_t p = il_position(l, (int64_t)(first + i));
        if (p < 0) return fail(NFEC_ENOTSUP, "npc: interleaver geometry the reference cannot map");
        pos[i] = (uint64_t)p;
    }
    return NFEC_OK;
}

int nfec_npc_encode_file(int device, const char* in_path, const char* out_path, const nfec_npc_params* p)
{
    const int32_t dev = device;
    return nfec_npc_encode_file_multi(&dev, 1, in_path, out_path, p);
}

int nfec_npc_encode_file_multi(const int32_t* devices, int32_t num_devices, const char* in_path, const char* out_path,
                               const nfec_npc_params* p)
{
    if (!in_path || !out_path || !p) return fail(NFEC_EINVAL, "null argument");
    int rc = check_devices(devices, num_devices);
    if (rc) return rc;
    Phases ph;
    MappedFile in;
    if ((rc = in.open_read(in_path))) return rc;
    ph.mark(4);
    nfec_npc_layout l;
    if ((rc = nfec_npc_layout_for(p, in.size, 1, &l))) return rc;
    const uint32_t k = l.num_data, m = l.num_parity, n = k + m;
    const uint32_t ss = l.segment_size, ds = ss - 4, stride = round8(ss);
    const uint64_t bstride = (uint64_t)n * stride;

    // the whole interleaver map first: a bad geometry fails before any output is written
    std::vector<uint64_t> pos(l.num_segments);
    if ((rc = nfec_npc_positions(&l, 0, l.num_segments, pos.data()))) return rc;
    ph.mark(5);

    // meta segment (normPrecode.cpp:650-678)
    std::vector<uint8_t> meta(ds, 0);
    for (int i = 0; i < 8; ++i) meta[i] = (uint8_t)(in.size >> (56 - 8 * i));
    const std::string name = base_name(in_path);
    std::memcpy(meta.data() + 8, name.data(), std::min<size_t>(name.size(), ss - 12));

    MappedFile out;
    if ((rc = out.open_write(out_path, l.num_segments * ss))) return rc;
    const bool zero_parity = l.kind == NFEC_RS16 && (ds & 1);  // RS16 leaves an odd last byte alone
    const uint32_t ndev = (uint32_t)std::min<uint64_t>((uint64_t)num_devices, l.num_blocks);
    const unsigned tpw = std::max(1u, Threads::total() / ndev);
    const uint32_t cb = chunk_blocks(bstride, (l.num_blocks + ndev - 1) / ndev);

    // one device's share: fill (host) -> H2D, encode, CRCs, D2H -> scatter (host), two staging
    // slots so the host copies of one chunk overlap the GPU work of the next
    auto worker = [&](uint32_t wi, int dev, uint64_t blo, uint64_t bhi) -> int {
        Phases* P = wi == 0 ? &ph : nullptr;
        Stage S;
        int rc = S.init(dev, l, stride, cb);
        if (rc) return rc;
        auto fill = [&](int slot, uint64_t b0, uint32_t nb) {
            uint8_t* H = S.hblk[slot];
            Threads::run(nb, tpw, [&](uint64_t lo, uint64_t hi) {
                for (uint64_t bi = lo; bi < hi; ++bi) {
                    const uint64_t b = b0 + bi;
                    const uint32_t nd = (b + 1 == l.num_blocks) ? l.last_block_data : k;
                    uint8_t* blk = H + bi * bstride;
                    if (nd < k) std::memset(blk, 0, (size_t)k * stride);
                    for (uint32_t i = 0; i < nd; ++i) {
                        const uint64_t j = b * k + i;  // input segment
                        uint8_t* dst = blk + (uint64_t)((b * m + i) % k) * stride;
                        if (j == 0) {
                            std::memcpy(dst, meta.data(), ds);
                        } else {
                            const uint32_t len = (j + 1 == l.input_segments) ? l.last_segment_bytes : ds;
                            std::memcpy(dst, in.p + (j - 1) * ds, len);
                            if (len < ds) std::memset(dst + len, 0, ds - len);
                        }
                    }
                }
            });
        };
        auto launch = [&](int slot, uint32_t nb) -> int {
            uint8_t* H = S.hblk[slot];
            NFEC_HIP(hipMemcpy2DAsync(S.dblk, bstride, H, bstride, (size_t)k * stride, nb, hipMemcpyHostToDevice, S.st));
            if (zero_parity)
                NFEC_HIP(hipMemset2DAsync(S.dblk + (size_t)k * stride, bstride, 0, (size_t)m * stride, nb, S.st));
            nfec_block_batch bb{};
            bb.blocks = S.dblk;
            bb.block_stride = bstride;
            bb.seg_stride = stride;
            bb.nblocks = nb;
            int r = nfec_encode(S.codec, &bb, S.st);
            if (r) return r;
            CrcArgs c;
            c.base = S.dblk;
            c.block_stride = bstride;
            c.seg_stride = stride;
            c.nblocks = nb;
            c.slots = n;
            c.len = ds;
            c.crc = S.dcrc;
            if ((r = launch_crc32_slots(c, S.st))) return r;
            NFEC_HIP(hipMemcpy2DAsync(H + (size_t)k * stride, bstride, S.dblk + (size_t)k * stride, bstride,
                                      (size_t)m * stride, nb, hipMemcpyDeviceToHost, S.st));
            NFEC_HIP(hipMemcpyAsync(S.hcrc[slot], S.dcrc, (size_t)nb * n * 4, hipMemcpyDeviceToHost, S.st));
            NFEC_HIP(hipEventRecord(S.done[slot], S.st));
            return NFEC_OK;
        };
        auto scatter = [&](int slot, uint64_t b0, uint32_t nb) -> int {
            NFEC_HIP(hipEventSynchronize(S.done[slot]));
            const uint8_t* H = S.hblk[slot];
            const uint32_t* crc = S.hcrc[slot];
            Threads::run(nb, tpw, [&](uint64_t lo, uint64_t hi) {
                for (uint64_t bi = lo; bi < hi; ++bi) {
                    const uint64_t b = b0 + bi;
                    const uint32_t nd = (b + 1 == l.num_blocks) ? l.last_block_data : k;
                    for (uint32_t t = 0; t < nd + m; ++t) {
                        const uint32_t s = t < nd ? (uint32_t)((b * m + t) % k) : k + (t - nd);
                        uint8_t* dst = out.p + pos[b * n + t] * ss;
                        std::memcpy(dst, H + bi * bstride + (uint64_t)s * stride, ds);
                        put_be32(dst + ds, crc[bi * n + s]);
                    }
                }
            });
            return NFEC_OK;
        };
        int slot = 0;
        uint64_t pb0 = 0;
        uint32_t pnb = 0;
        if (P) P->mark(0);
        for (uint64_t b0 = blo; b0 < bhi && !rc; b0 += cb) {
            const uint32_t nb = (uint32_t)std::min<uint64_t>(cb, bhi - b0);
            fill(slot, b0, nb);
            if (P) P->mark(1);
            // the staging slot being filled was last read by the scatter two chunks ago (host)
            if ((rc = launch(slot, nb))) break;
            if (P) P->mark(2);
            if (pnb) rc = scatter(slot ^ 1, pb0, pnb);
            if (P) P->mark(3);
            pb0 = b0;
            pnb = nb;
            slot ^= 1;
        }
        if (!rc && pnb) rc = scatter(slot ^ 1, pb0, pnb);
        if (P) P->mark(3);
        return rc;
    };
    rc = run_devices(devices, ndev, l.num_blocks, worker);
    ph.report("encode");
    return rc;
}

int nfec_npc_decode_file(int device, const char* in_path, const char* out_path, const nfec_npc_params* p,
                         uint64_t* out_bytes, char* name_out, size_t name_cap)
{
    const int32_t dev = device;
    return nfec_npc_decode_file_multi(&dev, 1, in_path, out_path, p, out_bytes, name_out, name_cap);
}

int nfec_npc_decode_file_multi(const int32_t* devices, int32_t num_devices, const char* in_path,
                               const char* out_path, const nfec_npc_params* p, uint64_t* out_bytes,
                               char* name_out, size_t name_cap)
{
    if (!in_path || !p) return fail(NFEC_EINVAL, "null argument");
    int rc = check_devices(devices, num_devices);
    if (rc) return rc;
    Phases ph;
    MappedFile in;
    if ((rc = in.open_read(in_path))) return rc;
    ph.mark(4);
    nfec_npc_layout l;
    if ((rc = nfec_npc_layout_for(p, in.size, 0, &l))) return rc;
    const uint32_t k = l.num_data, m = l.num_parity, n = k + m;
    const uint32_t ss = l.segment_size, ds = ss - 4, stride = round8(ss);
    const uint64_t bstride = (uint64_t)n * stride;
    std::vector<uint64_t> pos(l.num_segments);
    if ((rc = nfec_npc_positions(&l, 0, l.num_segments, pos.data()))) return rc;
    ph.mark(5);
    const uint32_t ndev = (uint32_t)std::min<uint64_t>((uint64_t)num_devices, l.num_blocks);
    const unsigned tpw = std::max(1u, Threads::total() / ndev);
    const uint32_t cb = chunk_blocks(bstride, (l.num_blocks + ndev - 1) / ndev);

    // The output's size and name are in the meta segment (block 0's first source segment), known
    // once block 0 is repaired: worker 0 opens the file then, the others wait for it before
    // their first write.  Block b's source lands at a fixed offset: every block before the last
    // holds k segments of ds bytes, and block 0's first is the meta segment.
    MappedFile outm;
    uint64_t out_size = 0;
    std::mutex omu;
    std::condition_variable ocv;
    int ostate = 0;  // 0 pending, 1 open, -1 worker 0 failed first
    std::atomic<uint64_t> written{0};
    auto out_offset = [&](uint64_t b) -> uint64_t { return b == 0 ? 0 : (b * k - 1) * ds; };
    auto seg_len = [&](uint64_t b, uint32_t i, uint32_t nd) -> uint32_t {
        if (b + 1 == l.num_blocks && i + 1 == nd) {
            const uint32_t len = (uint32_t)(out_size % ds);
            return len ? len : ds;
        }
        return ds;
    };
    auto set_state = [&](int st) {
        std::lock_guard<std::mutex> g(omu);
        if (ostate == 0) ostate = st;
        ocv.notify_all();
    };

    auto worker = [&](uint32_t wi, int dev, uint64_t blo, uint64_t bhi) -> int {
        Phases* P = wi == 0 ? &ph : nullptr;
        int rc = NFEC_OK;
        {
            Stage S;
            rc = S.init(dev, l, stride, cb);
            auto gather = [&](int slot, uint64_t b0, uint32_t nb) {
                uint8_t* H = S.hblk[slot];
                for (uint32_t bi = 0; bi < nb; ++bi)
                    S.hnd[slot][bi] = (uint16_t)((b0 + bi + 1 == l.num_blocks) ? l.last_block_data : k);
                Threads::run(nb, tpw, [&](uint64_t lo, uint64_t hi) {
                    for (uint64_t bi = lo; bi < hi; ++bi) {
                        const uint64_t b = b0 + bi;
                        const uint32_t nd = S.hnd[slot][bi];
                        for (uint32_t t = 0; t < nd + m; ++t)
                            std::memcpy(H + bi * bstride + (uint64_t)t * stride, in.p + pos[b * n + t] * ss, ss);
                    }
                });
            };
            auto launch = [&](int slot, uint32_t nb) -> int {
                uint8_t* H = S.hblk[slot];
                NFEC_HIP(hipMemcpyAsync(S.dblk, H, (size_t)nb * bstride, hipMemcpyHostToDevice, S.st));
                NFEC_HIP(hipMemcpyAsync(S.dnd, S.hnd[slot], (size_t)nb * 2, hipMemcpyHostToDevice, S.st));
                CrcArgs c;
                c.base = S.dblk;
                c.block_stride = bstride;
                c.seg_stride = stride;
                c.nblocks = nb;
                c.slots = n;
                c.len = ds;
                c.bad = S.dbad;
                int r;
                if ((r = launch_crc32_slots(c, S.st))) return r;
                ErasureListArgs e;
                e.bad = S.dbad;
                e.slots = n;
                e.num_data = S.dnd;
                e.k = k;
                e.m = m;
                e.nblocks = nb;
                e.locs = S.dlocs;
                e.stride = m;
                e.counts = S.dcounts;
                if ((r = launch_erasure_list(e, S.st))) return r;
                NFEC_HIP(hipMemcpyAsync(S.hcounts[slot], S.dcounts, (size_t)nb * 2, hipMemcpyDeviceToHost, S.st));
                NFEC_HIP(hipStreamSynchronize(S.st));
                for (uint32_t bi = 0; bi < nb; ++bi)
                    if (S.hcounts[slot][bi] > m)
                        return fail(NFEC_ERANGE, "npc: decoding encountered block with too many errors");
                // erased vectors are zeroed before Decode (normPrecode.cpp:1049, :1087)
                if ((r = launch_zero_slots(S.dblk, bstride, stride, nb, S.dlocs, m, S.dcounts, ds, S.st))) return r;
                nfec_block_batch bb{};
                bb.blocks = S.dblk;
                bb.block_stride = bstride;
                bb.seg_stride = stride;
                bb.nblocks = nb;
                bb.num_data = S.dnd;
                if ((r = nfec_decode(S.codec, &bb, S.dlocs, m, S.dcounts, S.dstatus, S.st))) return r;
                NFEC_HIP(hipMemcpy2DAsync(H, bstride, S.dblk, bstride, (size_t)k * stride, nb, hipMemcpyDeviceToHost, S.st));
                NFEC_HIP(hipEventRecord(S.done[slot], S.st));
                return NFEC_OK;
            };
            // write the source segments (normPrecode.cpp:1129-1175)
            auto emit = [&](int slot, uint64_t b0, uint32_t nb) -> int {
                NFEC_HIP(hipEventSynchronize(S.done[slot]));
                const uint8_t* H = S.hblk[slot];
                if (b0 == 0) {
                    const uint8_t* m0 = H;
                    uint64_t size = 0;
                    for (int i = 0; i < 8; ++i) size = (size << 8) | m0[i];
                    const size_t maxlen = std::min<size_t>(4096, ss - 12);
                    std::string nm(reinterpret_cast<const char*>(m0 + 8),
                                   strnlen(reinterpret_cast<const char*>(m0 + 8), maxlen));
                    if (name_out && name_cap) {
                        const size_t c = std::min(nm.size(), name_cap - 1);
                        std::memcpy(name_out, nm.data(), c);
                        name_out[c] = 0;
                    }
                    const std::string target = out_path ? std::string(out_path) : nm;
                    // every data segment but the meta one, the last cut to the file size (:1156-1161)
                    uint64_t total = 0;
                    if (l.input_segments >= 2) {
                        uint64_t last = size % ds;
                        if (last == 0) last = ds;
                        total = (l.input_segments - 2) * ds + last;
                    }
                    out_size = size;
                    const int r = outm.open_write(target.c_str(), total);
                    set_state(r ? -1 : 1);
                    if (r) return r;
                } else {
                    std::unique_lock<std::mutex> lk(omu);
                    ocv.wait(lk, [&] { return ostate != 0; });
                    if (ostate < 0) return NFEC_EINVAL;  // worker 0's error is the one reported
                }
                Threads::run(nb, tpw, [&](uint64_t lo, uint64_t hi) {
                    for (uint64_t bi = lo; bi < hi; ++bi) {
                        const uint64_t b = b0 + bi;
                        const uint32_t nd = S.hnd[slot][bi];
                        uint8_t* dst = outm.p + out_offset(b);
                        uint64_t bytes = 0;
                        for (uint32_t i = 0; i < nd; ++i) {
                            if (b == 0 && i == 0) continue;
                            const uint32_t len = seg_len(b, i, nd);
                            std::memcpy(dst, H + bi * bstride + (uint64_t)i * stride, len);
                            dst += len;
                            bytes += len;
                        }
                        written.fetch_add(bytes, std::memory_order_relaxed);
                    }
                });
                return NFEC_OK;
            };
            int slot = 0;
            uint64_t pb0 = 0;
            uint32_t pnb = 0;
            if (P) P->mark(0);
            for (uint64_t b0 = blo; b0 < bhi && !rc; b0 += cb) {
                const uint32_t nb = (uint32_t)std::min<uint64_t>(cb, bhi - b0);
                gather(slot, b0, nb);
                if (P) P->mark(1);
                if ((rc = launch(slot, nb))) break;
                if (P) P->mark(2);
                if (pnb) rc = emit(slot ^ 1, pb0, pnb);
                if (P) P->mark(3);
                pb0 = b0;
                pnb = nb;
                slot ^= 1;
            }
            if (!rc && pnb) rc = emit(slot ^ 1, pb0, pnb);
            if (P) P->mark(3);
        }
        // the output was never opened: release the workers waiting for it
        if (wi == 0) set_state(-1);
        return rc;
    };
    rc = run_devices(devices, ndev, l.num_blocks, worker);
    ph.report("decode");
    if (!rc && out_bytes) *out_bytes = written.load();
    return rc;
}

int nfec_crc32_slots(const nfec_block_batch* b, uint32_t slots, uint32_t len, uint32_t* crc, void* stream)
{
    if (!b || !b->blocks || !crc) return fail(NFEC_EINVAL, "null argument");
    if (len > b->seg_stride || (b->seg_stride & 7) || (b->block_stride & 7) ||
        (reinterpret_cast<uintptr_t>(b->blocks) & 7))
        return fail(NFEC_EINVAL, "crc32: len exceeds the segment stride or strides not 8-byte aligned");
    CrcArgs c;
    c.base = static_cast<const uint8_t*>(b->blocks);
    c.block_stride = b->block_stride;
    c.seg_stride = b->seg_stride;
    c.nblocks = b->nblocks;
    c.slots = slots;
    c.len = len;
    c.crc = crc;
    return launch_crc32_slots(c, static_cast<hipStream_t>(stream));
}

}  // extern "C"
