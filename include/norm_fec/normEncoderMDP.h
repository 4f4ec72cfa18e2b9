// normEncoderMDP.h -- GPU-backed NormEncoderMDP / NormDecoderMDP (the legacy MDP Reed-Solomon
// code, fec_id 129) under the reference's file name and include guard
// (include/normEncoderMDP.h:33-86).
//
// Included by name at normSession.cpp:3, normNode.cpp:4 and normPrecode.cpp:10.  Public surface
// = the reference's (normEncoderMDP.h:42-48, :66-72): Encode MUST be called in order of source
// vector 0, 1, 2, ... (one LFSR step per call, normEncoderMDP.cpp:178-211); Init requires
// numData + numParity <= 255; Decode treats missing vectors as zero (:333-430).
#ifndef _NORM_ENCODER_MDP
#define _NORM_ENCODER_MDP

#include "normEncoder.h"
#include "nfecCodecBase.h"

class NormEncoderMDP : public NormEncoder, public NfecCodecBase
{
  public:
    NormEncoderMDP();
    ~NormEncoderMDP();
    bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize);
    void Destroy();
    bool IsReady() { return codec != 0; }
    // "Encode" MUST be called in order of source vector0, vector1, vector2, etc
    void Encode(unsigned int segmentId, const char* dataVector, char** parityVectorList);

    unsigned int GetNumData() { return ndata; }
    unsigned int GetNumParity() { return npar; }
    unsigned int GetVectorSize() { return vector_size; }
};  // end class NormEncoderMDP

class NormDecoderMDP : public NormDecoder, public NfecCodecBase
{
  public:
    NormDecoderMDP();
    ~NormDecoderMDP();
    bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize);
    int Decode(char** vectorList, unsigned int numData, unsigned int erasureCount, unsigned int* erasureLocs);
    int NumParity() { return (int)npar; }
    int VectorSize() { return (int)vector_size; }
    void Destroy();

    unsigned int GetNumParity() { return npar; }
    unsigned int GetVectorSize() { return vector_size; }
};  // end class NormDecoderMDP

#endif  // _NORM_ENCODER_MDP
