// nfec_fectest.cpp -- the reference's FEC round-trip harness (src/common/fecTest.cpp:23-135),
// restated against the GPU drop-in classes and driven through NormEncoder* / NormDecoder*
// base-class pointers, the way NORM's engine holds its codecs (normSession.h:791,
// normNode.h:649).  Test infrastructure: built by tests/native/Makefile against libnfec.so
// only (plain g++, no HIP headers), run by tests/test_cxx_dropin.py on the GPU box and, with
// host-only codecs (no usable gfx950: the per-call paths on the CPU), in the CPU suite.
//
//   nfec_fectest KIND K M VEC NUMDATA IN OUT NULLPAR [LOC ...]
//     KIND     rs8 | rs16 | mdp
//     K M VEC  Init(numData=K, numParity=M, vectorSize=VEC)
//     NUMDATA  source segments actually coded (fecTest's SHORT_DATA; <= K)
//     IN       NUMDATA*VEC source bytes, or "-" for fecTest's printable data ('a' + i%26)
//     OUT      dump: encoded block (NUMDATA+M vectors), int32 Decode() return, repaired block
//     NULLPAR  1: erased parity passed as NULL pointers (NORM's receiver), 0: zeroed (fecTest)
//     LOC ...  sorted erasure locations in [0, NUMDATA+M)
// Exit status 0 when every source segment came back byte for byte (fecTest step 8).
//
// The codec headers are included exactly as NORM's construction sites include them
// (normSession.cpp:3-5), and tests/native/Makefile compiles this file with
// -I../../include/norm_fec ahead of poison/, a directory holding #error stand-ins under the
// reference's header names: it builds only if the engine's headers shadow the reference's.
// The inline accessors (GetNumData() & co., compiled here, not in the library) and sizeof()
// are checked against the library's own view of the classes (nfec_dropin_sizeof).
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "normEncoderMDP.h"  // "legacy" MDP Reed-Solomon encoder
#include "normEncoderRS8.h"  // 8-bit Reed-Solomon encoder of RFC 5510
#include "normEncoderRS16.h" // 16-bit Reed-Solomon encoder of RFC 5510

static int layout_errors = 0;

static void expect(bool ok, const char* what)
{
    if (!ok) {
        std::fprintf(stderr, "fect: %s\n", what);
        ++layout_errors;
    }
}

// new + Init through the concrete class, accessors read back, then handed out as the base
template <class E>
static NormEncoder* init_encoder(unsigned k, unsigned m, unsigned vec, int kind)
{
    E* e = new E;
    expect(sizeof(E) == nfec_dropin_sizeof(kind, 0), "encoder sizeof differs from the library's");
    if (!e->Init(k, m, (UINT16)vec)) {
        delete e;
        return 0;
    }
    expect(e->IsReady(), "encoder IsReady() false after Init");
    expect(e->GetNumData() == k && e->GetNumParity() == m && e->GetVectorSize() == vec,
           "encoder accessors do not return the Init parameters");
    return e;
}

template <class D>
static NormDecoder* init_decoder(unsigned k, unsigned m, unsigned vec, int kind)
{
    D* d = new D;
    expect(sizeof(D) == nfec_dropin_sizeof(kind, 1), "decoder sizeof differs from the library's");
    if (!d->Init(k, m, (UINT16)vec)) {
        delete d;
        return 0;
    }
    expect(d->GetNumParity() == m && d->GetVectorSize() == vec, "decoder accessors do not return the Init parameters");
    return d;
}

static NormEncoder* new_encoder(const char* kind, unsigned k, unsigned m, unsigned vec)
{
    if (!std::strcmp(kind, "rs8")) return init_encoder<NormEncoderRS8>(k, m, vec, NFEC_RS8);
    if (!std::strcmp(kind, "rs16")) return init_encoder<NormEncoderRS16>(k, m, vec, NFEC_RS16);
    if (!std::strcmp(kind, "mdp")) return init_encoder<NormEncoderMDP>(k, m, vec, NFEC_MDP);
    return 0;
}

static NormDecoder* new_decoder(const char* kind, unsigned k, unsigned m, unsigned vec)
{
    if (!std::strcmp(kind, "rs8")) return init_decoder<NormDecoderRS8>(k, m, vec, NFEC_RS8);
    if (!std::strcmp(kind, "rs16")) return init_decoder<NormDecoderRS16>(k, m, vec, NFEC_RS16);
    if (!std::strcmp(kind, "mdp")) {
        NormDecoder* d = init_decoder<NormDecoderMDP>(k, m, vec, NFEC_MDP);
        // the reference MDP decoder's own accessors (normEncoderMDP.h:70-71)
        if (d) expect(static_cast<NormDecoderMDP*>(d)->NumParity() == (int)m &&
                          static_cast<NormDecoderMDP*>(d)->VectorSize() == (int)vec,
                      "MDP decoder NumParity()/VectorSize() wrong");
        return d;
    }
    return 0;
}

// `nfec_fectest layout`: the sizeof() checks alone (no GPU needed)
static int layout_only()
{
    expect(sizeof(NormEncoderRS8) == nfec_dropin_sizeof(NFEC_RS8, 0), "NormEncoderRS8 sizeof differs");
    expect(sizeof(NormDecoderRS8) == nfec_dropin_sizeof(NFEC_RS8, 1), "NormDecoderRS8 sizeof differs");
    expect(sizeof(NormEncoderRS16) == nfec_dropin_sizeof(NFEC_RS16, 0), "NormEncoderRS16 sizeof differs");
    expect(sizeof(NormDecoderRS16) == nfec_dropin_sizeof(NFEC_RS16, 1), "NormDecoderRS16 sizeof differs");
    expect(sizeof(NormEncoderMDP) == nfec_dropin_sizeof(NFEC_MDP, 0), "NormEncoderMDP sizeof differs");
    expect(sizeof(NormDecoderMDP) == nfec_dropin_sizeof(NFEC_MDP, 1), "NormDecoderMDP sizeof differs");
    std::printf("layout %zu %zu %zu %zu %zu %zu errors %d\n", sizeof(NormEncoderRS8), sizeof(NormDecoderRS8),
                sizeof(NormEncoderRS16), sizeof(NormDecoderRS16), sizeof(NormEncoderMDP), sizeof(NormDecoderMDP),
                layout_errors);
    return layout_errors ? 1 : 0;
}

int main(int argc, char* argv[])
{
    if (argc == 2 && !std::strcmp(argv[1], "layout")) return layout_only();
    if (argc < 9) {
        std::fprintf(stderr, "usage: %s KIND K M VEC NUMDATA IN OUT NULLPAR [LOC ...]\n", argv[0]);
        return 2;
    }
    const char* kind = argv[1];
    const unsigned k = (unsigned)std::atoi(argv[2]), m = (unsigned)std::atoi(argv[3]);
    const unsigned vec = (unsigned)std::atoi(argv[4]), nd = (unsigned)std::atoi(argv[5]);
    const char* in_path = argv[6];
    const char* out_path = argv[7];
    const bool null_parity = std::atoi(argv[8]) != 0;
    std::vector<unsigned int> locs;
    for (int i = 9; i < argc; ++i) locs.push_back((unsigned)std::atoi(argv[i]));
    const unsigned n = nd + m;

    if (std::strcmp(kind, "rs8") && std::strcmp(kind, "rs16") && std::strcmp(kind, "mdp")) return 2;
    if (nd == 0 || nd > k) return 2;
    // NFEC_FECTEST_GPU=1: the per-call GPU round trips instead of the drop-in's host defaults
    if (const char* g = std::getenv("NFEC_FECTEST_GPU"))
        if (std::atoi(g) != 0) {
            NfecCodecBase::SetSegmentEncodeOnHost(false);
            NfecCodecBase::SetDecodeOnHost(false);
        }
    // NFEC_FECTEST_DEVICES=0,0,...: one codec striped over that device list (SetDevices, the
    // class-level route to nfec_codec_create_ex for a single NORM session's encoder)
    if (const char* dl = std::getenv("NFEC_FECTEST_DEVICES")) {
        int devs[NfecCodecBase::kMaxDevices], nd_ = 0;
        for (const char* p = dl; *p && nd_ < NfecCodecBase::kMaxDevices;) {
            devs[nd_++] = std::atoi(p);
            while (*p && *p != ',') ++p;
            if (*p == ',') ++p;
        }
        if (!NfecCodecBase::SetDevices(devs, nd_)) return 2;
    }
    NormEncoder* encoder = new_encoder(kind, k, m, vec);
    NormDecoder* decoder = new_decoder(kind, k, m, vec);
    if (!encoder || !decoder) {
        std::fprintf(stderr, "fect: Init(%u, %u, %u) failed\n", k, m, vec);
        return 3;
    }
    {
        // where the codecs live: host-only (no usable gfx950, NFEC_OPT_HOST_ONLY) or the GPU list
        NfecCodecBase* eb = dynamic_cast<NfecCodecBase*>(encoder);
        NfecCodecBase* db = dynamic_cast<NfecCodecBase*>(decoder);
        std::fprintf(stderr, "fect: host_only=%d/%d devices=%d/%d\n", eb->IsHostOnly() ? 1 : 0,
                     db->IsHostOnly() ? 1 : 0, nfec_codec_num_devices(eb->Handle(), 0, 0),
                     nfec_codec_num_devices(db->Handle(), 0, 0));
    }
    // Destroy / Init again through the vtable: Destroy must leave the codec reusable
    encoder->Destroy();
    if (!encoder->Init(k, m, (UINT16)vec)) return 3;

    // 1) source data, one heap allocation per segment (NORM's segment pool hands out
    //    scattered 8-byte-aligned buffers, normSegment.cpp:14-86)
    std::vector<char*> tx(n), rx(n);
    for (unsigned i = 0; i < n; ++i) {
        tx[i] = new char[vec];
        rx[i] = new char[vec];
    }
    if (!std::strcmp(in_path, "-")) {
        for (unsigned i = 0; i < nd; ++i) {
            std::memset(tx[i], 'a' + (i % 26), vec - 1);
            tx[i][vec - 1] = '\0';
        }
    } else {
        FILE* f = std::fopen(in_path, "rb");
        if (!f) return 2;
        for (unsigned i = 0; i < nd; ++i)
            if (std::fread(tx[i], 1, vec, f) != vec) return 2;
        std::fclose(f);
    }
    // 2) zero-init the parity vectors (the caller's contract, normObject.cpp:2240-2252)
    for (unsigned i = nd; i < n; ++i) std::memset(tx[i], 0, vec);
    // 3) encode one segment at a time, in order (MDP requires it)
    for (unsigned i = 0; i < nd; ++i) encoder->Encode(i, tx[i], tx.data() + nd);
    // 4) copy to the receive side
    for (unsigned i = 0; i < n; ++i) std::memcpy(rx[i], tx[i], vec);
    // 6) clear the erasures (erased source is zero-filled, normObject.cpp:1579)
    std::vector<char*> rxv(rx);
    for (unsigned loc : locs) {
        if (loc >= n) return 2;
        std::memset(rx[loc], 0, vec);
        if (null_parity && loc >= nd) rxv[loc] = 0;
    }
    // 7) decode
    const int status = decoder->Decode(rxv.data(), nd, (unsigned)locs.size(), locs.data());
    // 8) check decoding (RS16 codes vec/2 symbols: an odd last byte is never repaired,
    //    normEncoderRS16.cpp:733, so it is left out of the comparison)
    const unsigned cmp = std::strcmp(kind, "rs16") ? vec : (vec & ~1u);
    int bad = 0;
    for (unsigned i = 0; i < nd; ++i)
        if (std::memcmp(rx[i], tx[i], cmp)) {
            std::fprintf(stderr, "fect: segment:%u rxData decode error!\n", i);
            ++bad;
        }
    // dump for the oracle comparison
    FILE* f = std::fopen(out_path, "wb");
    if (!f) return 2;
    for (unsigned i = 0; i < n; ++i) std::fwrite(tx[i], 1, vec, f);
    std::fwrite(&status, sizeof(status), 1, f);
    for (unsigned i = 0; i < n; ++i) std::fwrite(rx[i], 1, vec, f);
    std::fclose(f);
    std::fprintf(stderr, "fect: %s k=%u m=%u vec=%u numData=%u erasures=%zu Decode()=%d bad=%d layout_errors=%d\n",
                 kind, k, m, vec, nd, locs.size(), status, bad, layout_errors);
    for (unsigned i = 0; i < n; ++i) {
        delete[] tx[i];
        delete[] rx[i];
    }
    delete encoder;  // through the base class: the virtual destructors release the GPU codec
    delete decoder;
    return (bad || layout_errors) ? 1 : 0;
}
