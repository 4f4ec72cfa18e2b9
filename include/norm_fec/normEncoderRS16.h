// normEncoderRS16.h -- GPU-backed NormEncoderRS16 / NormDecoderRS16 (16-bit Reed-Solomon of
// RFC 5510) under the reference's file name and include guard (include/normEncoderRS16.h:1-68).
//
// Included by name at normSession.cpp:5, normNode.cpp:6 and normPrecode.cpp:13.  Public surface
// = the reference's (normEncoderRS16.h:10-22, :37-46); Init accepts numData + numParity <=
// 65535, the code works on vectorSize/2 native-endian 16-bit symbols and never writes an odd
// last byte (normEncoderRS16.cpp:472-482, :733).
#ifndef _NORM_ENCODER_RS16
#define _NORM_ENCODER_RS16

#include "normEncoder.h"
#include "nfecCodecBase.h"

class NormEncoderRS16 : public NormEncoder, public NfecCodecBase
{
  public:
    NormEncoderRS16();
    ~NormEncoderRS16();

    virtual bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize);
    virtual void Destroy();
    virtual void Encode(unsigned int segmentId, const char* dataVector, char** parityVectorList);

    unsigned int GetNumData() { return ndata; }
    unsigned int GetNumParity() { return npar; }
    unsigned int GetVectorSize() { return vector_size; }
    bool IsReady() { return codec != 0; }
};  // end class NormEncoderRS16

class NormDecoderRS16 : public NormDecoder, public NfecCodecBase
{
  public:
    NormDecoderRS16();
    virtual ~NormDecoderRS16();
    virtual bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize);
    virtual void Destroy();
    virtual int Decode(char** vectorList, unsigned int numData, unsigned int erasureCount,
                       unsigned int* erasureLocs);

    unsigned int GetNumParity() { return npar; }
    unsigned int GetVectorSize() { return vector_size; }
};  // end class NormDecoderRS16

#endif  // _NORM_ENCODER_RS16
