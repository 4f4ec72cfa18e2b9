// nfec_fectest.cpp -- the reference's FEC round-trip harness (src/common/fecTest.cpp:23-135),
// restated against the GPU drop-in classes and driven through NormEncoder* / NormDecoder*
// base-class pointers, the way NORM's engine holds its codecs (normSession.h:791,
// normNode.h:649).  Test infrastructure: built by tests/native/Makefile against libnfec.so
// only (plain g++, no HIP headers), run by tests/test_cxx_dropin.py on the GPU box.
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
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "norm_fec/nfecCodecs.h"

static NormEncoder* new_encoder(const char* kind)
{
    if (!std::strcmp(kind, "rs8")) return new NormEncoderRS8;
    if (!std::strcmp(kind, "rs16")) return new NormEncoderRS16;
    if (!std::strcmp(kind, "mdp")) return new NormEncoderMDP;
    return 0;
}

static NormDecoder* new_decoder(const char* kind)
{
    if (!std::strcmp(kind, "rs8")) return new NormDecoderRS8;
    if (!std::strcmp(kind, "rs16")) return new NormDecoderRS16;
    if (!std::strcmp(kind, "mdp")) return new NormDecoderMDP;
    return 0;
}

int main(int argc, char* argv[])
{
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

    NormEncoder* encoder = new_encoder(kind);
    NormDecoder* decoder = new_decoder(kind);
    if (!encoder || !decoder || nd == 0 || nd > k) return 2;
    // Init / Destroy / Init again through the vtable: Destroy must leave the codec reusable
    if (!encoder->Init(k, m, (UINT16)vec) || !decoder->Init(k, m, (UINT16)vec)) {
        std::fprintf(stderr, "fect: Init(%u, %u, %u) failed\n", k, m, vec);
        return 3;
    }
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
    std::fprintf(stderr, "fect: %s k=%u m=%u vec=%u numData=%u erasures=%zu Decode()=%d bad=%d\n", kind, k, m, vec,
                 nd, locs.size(), status, bad);
    for (unsigned i = 0; i < n; ++i) {
        delete[] tx[i];
        delete[] rx[i];
    }
    delete encoder;  // through the base class: the virtual destructors release the GPU codec
    delete decoder;
    return bad ? 1 : 0;
}
