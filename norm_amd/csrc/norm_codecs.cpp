// norm_codecs.cpp -- NormEncoder/NormDecoder drop-in classes over the nfec C ABI.
//
// Compiled from the reference-named headers (include/norm_fec/normEncoder*.h), exactly the
// include lines of NORM's construction sites (normSession.cpp:3-5, normNode.cpp:4-6), so the
// library and a NORM translation unit see one class layout.
#include "../../include/norm_fec/normEncoderMDP.h"
#include "../../include/norm_fec/normEncoderRS8.h"
#include "../../include/norm_fec/normEncoderRS16.h"

#include <cstdio>

NormEncoder::~NormEncoder() {}
NormDecoder::~NormDecoder() {}

int NfecCodecBase::default_device = 0;
int NfecCodecBase::device_list[NfecCodecBase::kMaxDevices] = {};
int NfecCodecBase::num_devices = 0;
bool NfecCodecBase::segment_on_host = true;
bool NfecCodecBase::decode_on_host = true;
bool NfecCodecBase::host_fallback = true;
bool NfecCodecBase::devices_chosen = false;

bool NfecCodecBase::SetDevices(const int* devices, int count)
{
    if (count < 1 || count > kMaxDevices || !devices) return false;
    default_device = devices[0];
    num_devices = count > 1 ? count : 0;
    devices_chosen = true;
    for (int i = 0; i < count; ++i) device_list[i] = devices[i];
    return true;
}

int NfecCodecBase::GetDevices(int* devices, int cap)
{
    const int n = num_devices ? num_devices : 1;
    for (int i = 0; devices && i < n && i < cap; ++i) devices[i] = num_devices ? device_list[i] : default_device;
    return n;
}

bool NfecCodecBase::IsHostOnly() const
{
    nfec_codec_info info;
    return codec && nfec_codec_get_info(codec, &info) == NFEC_OK && info.device < 0;
}

bool NfecCodecBase::InitCodec(int kind, unsigned int numData, unsigned int numParity, UINT16 vectorSize)
{
    DestroyCodec();
    nfec_codec* c = 0;
    nfec_codec_config cfg;
    cfg.kind = kind;
    cfg.num_data = numData;
    cfg.num_parity = numParity;
    cfg.vector_size = vectorSize;
    int32_t devs[kMaxDevices];
    const int n = num_devices ? num_devices : 1;
    for (int i = 0; i < n; ++i) devs[i] = num_devices ? device_list[i] : default_device;
    cfg.devices = devs;
    cfg.num_devices = (uint32_t)n;
    cfg.flags = 0;
    int rc = nfec_codec_create_ex(&cfg, &c);
    if (rc == NFEC_EDEVICE && host_fallback && segment_on_host && decode_on_host && !devices_chosen &&
        nfec_device_count() == 0) {
        // no usable gfx950 in this process and none asked for: a host-only codec still serves
        // NORM's per-call Encode / Decode (a bad device choice or a failure on a present GPU is
        // an Init failure instead, below)
        cfg.devices = 0;
        cfg.num_devices = 0;
        cfg.flags = NFEC_OPT_HOST_ONLY;
        rc = nfec_codec_create_ex(&cfg, &c);
        if (rc == NFEC_OK)
            std::fprintf(stderr, "nfec: no usable gfx950 device: Init(%u, %u, %u) built a host-only codec "
                                 "(per-call Encode / Decode on the CPU)\n",
                         numData, numParity, (unsigned)vectorSize);
    }
    if (rc != NFEC_OK) {
        // the reference logs PL_FATAL and returns false (normEncoderRS8.cpp:405-409)
        std::fprintf(stderr, "nfec: Init(%u, %u, %u) failed: %s\n", numData, numParity, (unsigned)vectorSize,
                     nfec_last_error());
        return false;
    }
    codec = c;
    ndata = numData;
    npar = numParity;
    vector_size = vectorSize;
    return true;
}

void NfecCodecBase::DestroyCodec()
{
    if (codec) nfec_codec_destroy(codec);
    codec = 0;
    ndata = npar = vector_size = 0;
}

int NfecCodecBase::EncodeBlocks(const nfec_block_batch* batch, void* stream)
{
    return codec ? nfec_encode(codec, batch, stream) : NFEC_EINVAL;
}

int NfecCodecBase::DecodeBlocks(const nfec_block_batch* batch, const uint16_t* erasureLocs, uint32_t erasureStride,
                                const uint16_t* erasureCounts, int32_t* status, void* stream)
{
    return codec ? nfec_decode(codec, batch, erasureLocs, erasureStride, erasureCounts, status, stream)
                 : NFEC_EINVAL;
}

#define NFEC_DEFINE_ENCODER(NAME, KIND)                                                          \
    NAME::NAME() {}                                                                              \
    NAME::~NAME() { DestroyCodec(); }                                                            \
    bool NAME::Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize)             \
    {                                                                                            \
        return InitCodec(KIND, numData, numParity, vectorSize);                                  \
    }                                                                                            \
    void NAME::Destroy() { DestroyCodec(); }                                                     \
    void NAME::Encode(unsigned int segmentId, const char* dataVector, char** parityVectorList)   \
    {                                                                                            \
        if (!codec) return;                                                                      \
        int rc = segment_on_host                                                                 \
                     ? nfec_encode_segment_host(codec, segmentId, dataVector, (void* const*)parityVectorList) \
                     : nfec_encode_segment(codec, segmentId, dataVector, (void* const*)parityVectorList); \
        if (rc != NFEC_OK) std::fprintf(stderr, "nfec: Encode failed: %s\n", nfec_last_error()); \
    }

#define NFEC_DEFINE_DECODER(NAME, KIND)                                                          \
    NAME::NAME() {}                                                                              \
    NAME::~NAME() { DestroyCodec(); }                                                            \
    bool NAME::Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize)             \
    {                                                                                            \
        return InitCodec(KIND, numData, numParity, vectorSize);                                  \
    }                                                                                            \
    void NAME::Destroy() { DestroyCodec(); }                                                     \
    int NAME::Decode(char** vectorList, unsigned int numData, unsigned int erasureCount,         \
                     unsigned int* erasureLocs)                                                  \
    {                                                                                            \
        if (!codec) return 0;                                                                    \
        int rc = (decode_on_host && nfec_decode_host_preferred(codec, numData, erasureCount))    \
                     ? nfec_decode_vectors_host(codec, (void* const*)vectorList, numData, erasureCount, \
                                                (const uint32_t*)erasureLocs)                    \
                     : nfec_decode_vectors(codec, (void* const*)vectorList, numData, erasureCount, \
                                           (const uint32_t*)erasureLocs);                        \
        if (rc < 0) {                                                                            \
            std::fprintf(stderr, "nfec: Decode failed: %s\n", nfec_last_error());                \
            return 0;                                                                            \
        }                                                                                        \
        return rc;                                                                               \
    }

NFEC_DEFINE_ENCODER(NormEncoderRS8, NFEC_RS8)
NFEC_DEFINE_DECODER(NormDecoderRS8, NFEC_RS8)
NFEC_DEFINE_ENCODER(NormEncoderRS16, NFEC_RS16)
NFEC_DEFINE_DECODER(NormDecoderRS16, NFEC_RS16)
NFEC_DEFINE_ENCODER(NormEncoderMDP, NFEC_MDP)
NFEC_DEFINE_DECODER(NormDecoderMDP, NFEC_MDP)

extern "C" size_t nfec_dropin_sizeof(int kind, int decoder)
{
    switch (kind) {
        case NFEC_RS8: return decoder ? sizeof(NormDecoderRS8) : sizeof(NormEncoderRS8);
        case NFEC_RS16: return decoder ? sizeof(NormDecoderRS16) : sizeof(NormEncoderRS16);
        case NFEC_MDP: return decoder ? sizeof(NormDecoderMDP) : sizeof(NormEncoderMDP);
        default: return 0;
    }
}
