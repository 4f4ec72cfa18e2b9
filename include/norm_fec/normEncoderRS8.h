// normEncoderRS8.h -- GPU-backed NormEncoderRS8 / NormDecoderRS8 (8-bit Reed-Solomon of
// RFC 5510) under the reference's file name and include guard (include/normEncoderRS8.h:1-69).
//
// NORM's construction sites include this file by name (normSession.cpp:4, normNode.cpp:5,
// normPrecode.cpp:12) and call new NormEncoderRS8 / new NormDecoderRS8; with
// -I<nfec>/include/norm_fec ahead of NORM's include/ they compile against these declarations,
// which the library's constructors and methods were compiled from too.
// Public surface = the reference's (normEncoderRS8.h:10-22, :36-45):
//   Init   -> false when numData + numParity > 255; without a usable gfx950 device it builds a
//             host-only codec (per-call Encode / Decode on the CPU; NfecCodecBase::SetHostFallback)
//   Encode -> parity_i ^= G[k+i][segmentId] * data (normEncoderRS8.cpp:473-483)
//   Decode -> erasureCount on success, 0 when the block cannot be repaired (:652-757)
// Calls go through include/nfec.h and are synchronous.  Batches run on the GPU; the per-call
// Encode / Decode run on the host CPU by default (NfecCodecBase::SetSegmentEncodeOnHost /
// SetDecodeOnHost select the GPU round trip instead).
#ifndef _NORM_ENCODER_RS8
#define _NORM_ENCODER_RS8

#include "normEncoder.h"
#include "nfecCodecBase.h"

class NormEncoderRS8 : public NormEncoder, public NfecCodecBase
{
  public:
    NormEncoderRS8();
    ~NormEncoderRS8();

    virtual bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize);
    virtual void Destroy();
    virtual void Encode(unsigned int segmentId, const char* dataVector, char** parityVectorList);

    unsigned int GetNumData() { return ndata; }
    unsigned int GetNumParity() { return npar; }
    unsigned int GetVectorSize() { return vector_size; }
    bool IsReady() { return codec != 0; }
};  // end class NormEncoderRS8

class NormDecoderRS8 : public NormDecoder, public NfecCodecBase
{
  public:
    NormDecoderRS8();
    virtual ~NormDecoderRS8();
    virtual bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize);
    virtual void Destroy();
    virtual int Decode(char** vectorList, unsigned int numData, unsigned int erasureCount,
                       unsigned int* erasureLocs);

    unsigned int GetNumParity() { return npar; }
    unsigned int GetVectorSize() { return vector_size; }
};  // end class NormDecoderRS8

#endif  // _NORM_ENCODER_RS8
