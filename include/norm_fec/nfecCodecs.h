// nfecCodecs.h -- GPU-backed drop-ins for NormEncoderRS8/RS16/MDP and NormDecoderRS8/RS16/MDP.
//
// Method names, argument meaning, return values and accessors follow the reference
// (include/normEncoderRS8.h:9-66, normEncoderRS16.h:9-65, normEncoderMDP.h:38-84):
//   Init  -> false on k+m beyond the field or when no gfx950 device is usable
//   Encode-> parity_i ^= G[k+i][segmentId] * data (RS), one in-order LFSR step (MDP)
//   Decode-> erasureCount on success, 0 if the block cannot be repaired
// Every call runs on the GPU through include/nfec.h.  Per-call Encode/Decode are
// synchronous round trips (correct but latency-bound); the batch methods EncodeBlocks /
// DecodeBlocks are the throughput path for block-at-once call sites such as
// NormObject::CalculateBlockParity (src/common/normObject.cpp:2203-2229).
#ifndef NFEC_CODECS_H
#define NFEC_CODECS_H

#include "normEncoder.h"
#include "../nfec.h"

class NfecCodecBase
{
  public:
    static void SetDevice(int device) { default_device = device; }
    static int GetDevice() { return default_device; }
    nfec_codec* Handle() const { return codec; }
    // Batched device-resident calls (see nfec_encode / nfec_decode).
    int EncodeBlocks(const nfec_block_batch* batch, void* stream);
    int DecodeBlocks(const nfec_block_batch* batch, const uint16_t* erasureLocs, uint32_t erasureStride,
                     const uint16_t* erasureCounts, int32_t* status, void* stream);

  protected:
    NfecCodecBase() : codec(0), ndata(0), npar(0), vector_size(0) {}
    bool InitCodec(int kind, unsigned int numData, unsigned int numParity, UINT16 vectorSize);
    void DestroyCodec();
    nfec_codec* codec;
    unsigned int ndata, npar, vector_size;
    static int default_device;
};

#define NFEC_DECLARE_ENCODER(NAME)                                                              \
    class NAME : public NormEncoder, public NfecCodecBase                                        \
    {                                                                                            \
      public:                                                                                    \
        NAME();                                                                                  \
        ~NAME();                                                                                 \
        virtual bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize);      \
        virtual void Destroy();                                                                  \
        virtual void Encode(unsigned int segmentId, const char* dataVector, char** parityVectorList); \
        unsigned int GetNumData() { return ndata; }                                              \
        unsigned int GetNumParity() { return npar; }                                             \
        unsigned int GetVectorSize() { return vector_size; }                                     \
        bool IsReady() { return codec != 0; }                                                    \
    };

#define NFEC_DECLARE_DECODER(NAME)                                                              \
    class NAME : public NormDecoder, public NfecCodecBase                                        \
    {                                                                                            \
      public:                                                                                    \
        NAME();                                                                                  \
        virtual ~NAME();                                                                         \
        virtual bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize);      \
        virtual void Destroy();                                                                  \
        virtual int Decode(char** vectorList, unsigned int numData, unsigned int erasureCount,   \
                           unsigned int* erasureLocs);                                           \
        unsigned int GetNumParity() { return npar; }                                             \
        unsigned int GetVectorSize() { return vector_size; }                                     \
        int NumParity() { return (int)npar; }                                                    \
        int VectorSize() { return (int)vector_size; }                                            \
    };

NFEC_DECLARE_ENCODER(NormEncoderRS8)
NFEC_DECLARE_DECODER(NormDecoderRS8)
NFEC_DECLARE_ENCODER(NormEncoderRS16)
NFEC_DECLARE_DECODER(NormDecoderRS16)
NFEC_DECLARE_ENCODER(NormEncoderMDP)
NFEC_DECLARE_DECODER(NormDecoderMDP)

#endif
