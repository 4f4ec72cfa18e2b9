// percall.cpp -- per-call latency of the drop-in classes (NORM's incremental sender path and
// one-block receiver repair) next to the oracle's CPU restatement of the reference codec.
//
//   percall KIND K M VEC ERASURES ITERS      KIND: rs8 | rs16 | mdp
//
// Encode: the sender's per-segment call (normObject.cpp:2038-2052 -> NormEncoderRS8::Encode,
// normEncoderRS8.cpp:473-483), cycling segmentId over 0..K-1 into zeroed parity.
// Decode: one block, ERASURES source erasures (zero-filled, normObject.cpp:1579), through
// NormDecoder::Decode (normEncoderRS8.cpp:652-757): the default path, the GPU round trip and
// the host path.  Prints one JSON line of microseconds per
// call.  Built against libnfec.so (the drop-in headers, as NORM includes them) and the oracle
// library (test infrastructure; its timing is the CPU reference per call).
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <vector>

#include "normEncoderMDP.h"
#include "normEncoderRS8.h"
#include "normEncoderRS16.h"

extern "C" {
int orc_rs8_generator(unsigned k, unsigned m, uint8_t* enc_out);
int orc_rs16_generator(unsigned k, unsigned m, uint16_t* enc_out);
void orc_rs8_encode(const uint8_t* enc, unsigned k, unsigned m, unsigned vec, unsigned segment_id,
                    const uint8_t* data, uint8_t** parity);
void orc_rs16_encode(const uint16_t* enc, unsigned k, unsigned m, unsigned vec, unsigned segment_id,
                     const uint8_t* data, uint8_t** parity);
int orc_rs8_decode(const uint8_t* enc, unsigned k, unsigned m, unsigned vec, uint8_t** vectors, unsigned num_data,
                   unsigned erasure_count, const unsigned* erasure_locs);
int orc_rs16_decode(const uint16_t* enc, unsigned k, unsigned m, unsigned vec, uint8_t** vectors,
                    unsigned num_data, unsigned erasure_count, const unsigned* erasure_locs);
int orc_mdp_generator_poly(unsigned m, uint8_t* g);
void orc_mdp_encode(const uint8_t* g, unsigned m, unsigned vec, const uint8_t* data, uint8_t** parity, uint8_t* scratch);
int orc_mdp_decode(unsigned m, unsigned vec, uint8_t** dvec, unsigned num_data, unsigned erasure_count,
                   const unsigned* locs);
}

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv)
{
    if (argc < 7) {
        std::fprintf(stderr, "usage: %s KIND K M VEC ERASURES ITERS\n", argv[0]);
        return 2;
    }
    const char* kind = argv[1];
    const unsigned k = std::atoi(argv[2]), m = std::atoi(argv[3]), vec = std::atoi(argv[4]);
    const unsigned ne = std::atoi(argv[5]), iters = std::atoi(argv[6]);
    const bool rs16 = !std::strcmp(kind, "rs16"), mdp = !std::strcmp(kind, "mdp");
    NormEncoder* enc = rs16 ? (NormEncoder*)new NormEncoderRS16 : mdp ? (NormEncoder*)new NormEncoderMDP
                                                                       : (NormEncoder*)new NormEncoderRS8;
    NormDecoder* dec = rs16 ? (NormDecoder*)new NormDecoderRS16 : mdp ? (NormDecoder*)new NormDecoderMDP
                                                                       : (NormDecoder*)new NormDecoderRS8;
    if (!enc->Init(k, m, (UINT16)vec) || !dec->Init(k, m, (UINT16)vec)) return 3;
    const unsigned n = k + m;
    std::vector<std::vector<char>> seg(n, std::vector<char>(vec));
    srand(7);
    for (unsigned i = 0; i < k; ++i)
        for (unsigned j = 0; j < vec; ++j) seg[i][j] = (char)rand();
    std::vector<char*> list(n);
    for (unsigned i = 0; i < n; ++i) list[i] = seg[i].data();

    // ---- per-segment Encode ----
    for (unsigned p = k; p < n; ++p) std::memset(list[p], 0, vec);
    for (unsigned i = 0; i < 8; ++i) enc->Encode(i % k, list[i % k], list.data() + k);  // warm-up
    for (unsigned p = k; p < n; ++p) std::memset(list[p], 0, vec);
    double t0 = now_us();
    for (unsigned i = 0; i < iters; ++i) enc->Encode(i % k, list[i % k], list.data() + k);
    const double enc_us = (now_us() - t0) / iters;
    // Encode runs on the host CPU by default (nfec_encode_segment_host); the GPU round trip
    // (nfec_encode_segment) beside it
    double enc_gpu_us = -1;
    {
        NfecCodecBase::SetSegmentEncodeOnHost(false);
        for (unsigned i = 0; i < 8; ++i) enc->Encode(i % k, list[i % k], list.data() + k);
        t0 = now_us();
        for (unsigned i = 0; i < iters; ++i) enc->Encode(i % k, list[i % k], list.data() + k);
        enc_gpu_us = (now_us() - t0) / iters;
        NfecCodecBase::SetSegmentEncodeOnHost(true);
    }
    // a clean encode of the block for the decode below
    for (unsigned p = k; p < n; ++p) std::memset(list[p], 0, vec);
    for (unsigned i = 0; i < k; ++i) enc->Encode(i, list[i], list.data() + k);
    std::vector<std::vector<char>> parity_dropin(m);
    for (unsigned p = 0; p < m; ++p) parity_dropin[p] = seg[k + p];

    // ---- one-block Decode with ne source erasures ----
    std::vector<unsigned> locs;
    for (unsigned i = 0; i < ne; ++i) locs.push_back(i * (k / (ne ? ne : 1)));
    std::vector<std::vector<char>> keep(ne);
    for (unsigned i = 0; i < ne; ++i) keep[i] = seg[locs[i]];
    int bad = 0, st = 0;
    auto time_decode = [&](const std::function<int()>& call) {
        double us = 0;
        for (unsigned it = 0; it < iters + 2; ++it) {
            for (unsigned i = 0; i < ne; ++i) std::memset(list[locs[i]], 0, vec);
            const double t = now_us();
            st = call();
            if (it >= 2) us += now_us() - t;
            for (unsigned i = 0; i < ne; ++i)
                bad += std::memcmp(list[locs[i]], keep[i].data(), rs16 ? vec & ~1u : vec) != 0;
        }
        return us / iters;
    };
    auto drop_in = [&]() { return dec->Decode(list.data(), k, ne, locs.data()); };
    // Decode's default path (the drop-in's policy, nfec_decode_host_preferred), the GPU round
    // trip (nfec_decode_vectors) and the host path (nfec_decode_vectors_host) beside it
    NfecCodecBase* dbase = dynamic_cast<NfecCodecBase*>(dec);
    const bool dec_host = dbase && nfec_decode_host_preferred(dbase->Handle(), k, ne) == 1;
    const double dec_us = time_decode(drop_in);
    NfecCodecBase::SetDecodeOnHost(false);
    const double dec_gpu_us = time_decode(drop_in);
    NfecCodecBase::SetDecodeOnHost(true);
    double dec_host_us = -1;
    if (dbase && nfec_decode_vectors_host(dbase->Handle(), (void* const*)list.data(), k, ne, locs.data()) >= 0)
        dec_host_us = time_decode([&]() {
            return nfec_decode_vectors_host(dbase->Handle(), (void* const*)list.data(), k, ne, locs.data());
        });

    // ---- the oracle (CPU restatement of the reference codec), same calls ----
    double orc_enc_us = -1, orc_dec_us = -1;
    if (!mdp) {
        std::vector<uint16_t> g16(rs16 ? (size_t)n * k : 1);
        std::vector<uint8_t> g8(rs16 ? 1 : (size_t)n * k);
        if (rs16) orc_rs16_generator(k, m, g16.data());
        else orc_rs8_generator(k, m, g8.data());
        uint8_t** ul = reinterpret_cast<uint8_t**>(list.data());
        const unsigned oit = iters * 4;
        t0 = now_us();
        for (unsigned i = 0; i < oit; ++i) {
            if (rs16) orc_rs16_encode(g16.data(), k, m, vec, i % k, ul[i % k], ul + k);
            else orc_rs8_encode(g8.data(), k, m, vec, i % k, ul[i % k], ul + k);
        }
        orc_enc_us = (now_us() - t0) / oit;
        for (unsigned p = k; p < n; ++p) std::memset(list[p], 0, vec);
        for (unsigned i = 0; i < k; ++i) {
            if (rs16) orc_rs16_encode(g16.data(), k, m, vec, i, ul[i], ul + k);
            else orc_rs8_encode(g8.data(), k, m, vec, i, ul[i], ul + k);
        }
        // the drop-in's parity equals the oracle's
        for (unsigned p = 0; p < m; ++p) bad += std::memcmp(parity_dropin[p].data(), list[k + p], vec) != 0;
        orc_dec_us = 0;
        for (unsigned it = 0; it < iters; ++it) {
            for (unsigned i = 0; i < ne; ++i) std::memset(list[locs[i]], 0, vec);
            const double t = now_us();
            if (rs16) orc_rs16_decode(g16.data(), k, m, vec, ul, k, ne, locs.data());
            else orc_rs8_decode(g8.data(), k, m, vec, ul, k, ne, locs.data());
            orc_dec_us += now_us() - t;
        }
        orc_dec_us /= iters;
    } else {
        // MDP: the reference's in-order LFSR Encode and syndrome / Forney Decode
        std::vector<uint8_t> g(m + 1), scratch(vec);
        orc_mdp_generator_poly(m, g.data());
        uint8_t** ul = reinterpret_cast<uint8_t**>(list.data());
        const unsigned oit = iters * 4;
        t0 = now_us();
        for (unsigned i = 0; i < oit; ++i) orc_mdp_encode(g.data(), m, vec, ul[i % k], ul + k, scratch.data());
        orc_enc_us = (now_us() - t0) / oit;
        for (unsigned p = k; p < n; ++p) std::memset(list[p], 0, vec);
        for (unsigned i = 0; i < k; ++i) orc_mdp_encode(g.data(), m, vec, ul[i], ul + k, scratch.data());
        for (unsigned p = 0; p < m; ++p) bad += std::memcmp(parity_dropin[p].data(), list[k + p], vec) != 0;
        orc_dec_us = 0;
        for (unsigned it = 0; it < iters; ++it) {
            for (unsigned i = 0; i < ne; ++i) std::memset(list[locs[i]], 0, vec);
            const double t = now_us();
            orc_mdp_decode(m, vec, ul, k, ne, locs.data());
            orc_dec_us += now_us() - t;
        }
        orc_dec_us /= iters;
        for (unsigned i = 0; i < ne; ++i) bad += std::memcmp(list[locs[i]], keep[i].data(), vec) != 0;
    }
    std::printf("{\"kind\": \"%s\", \"k\": %u, \"m\": %u, \"vec\": %u, \"erasures\": %u, \"iters\": %u, "
                "\"encode_us_per_call\": %.2f, \"encode_gpu_us_per_call\": %.2f, \"encode_path\": \"%s\", "
                "\"decode_us_per_call\": %.2f, \"decode_gpu_us_per_call\": %.2f, \"decode_host_us_per_call\": %.2f, "
                "\"decode_path\": \"%s\", "
                "\"decode_status\": %d, \"bad\": %d, "
                "\"oracle_encode_us_per_call\": %.2f, \"oracle_decode_us_per_call\": %.2f}\n",
                kind, k, m, vec, ne, iters, enc_us, enc_gpu_us,
                "host (nfec_encode_segment_host)", dec_us, dec_gpu_us, dec_host_us,
                dec_host ? "host (nfec_decode_vectors_host)" : "gpu (nfec_decode_vectors)", st, bad,
                orc_enc_us, orc_dec_us);
    delete enc;
    delete dec;
    return bad ? 1 : 0;
}
