// normEncoder.h -- NormEncoder / NormDecoder plugin surface for the MI355X FEC engine.
//
// Replaces the reference's include/normEncoder.h (abstract bases at normEncoder.h:38-54) under
// the same file name and the same include guard, so a NORM tree compiled with
// -I<nfec>/include/norm_fec ahead of its own include/ picks this header up wherever it writes
// #include "normEncoder.h" (normSession.h:7, normObject.h:5, normNode.h:6 and the codec headers),
// and never sees a second definition of these classes.  The declarations are token-for-token
// the reference's.
#ifndef _NORM_ENCODER
#define _NORM_ENCODER

// Inside a NORM tree protolib supplies UINT8/UINT16/UINT32 (the reference includes protokit.h
// here, normEncoder.h:36); standalone builds (the tests, a non-NORM host) get the same types.
#if defined(NFEC_WITH_PROTOLIB)
#include "protokit.h"
#elif defined(__has_include)
#if __has_include("protokit.h")
#include "protokit.h"
#define NFEC_WITH_PROTOLIB 1
#endif
#endif
#ifndef NFEC_WITH_PROTOLIB
#include <stdint.h>
typedef uint8_t UINT8;
typedef uint16_t UINT16;
typedef uint32_t UINT32;
#endif

class NormEncoder
{
  public:
    virtual ~NormEncoder();
    virtual bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize) = 0;
    virtual void Destroy() = 0;
    virtual void Encode(unsigned int segmentId, const char* dataVector, char** parityVectorList) = 0;
};  // end class NormEncoder

class NormDecoder
{
  public:
    virtual ~NormDecoder();
    virtual bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize) = 0;
    virtual void Destroy() = 0;
    virtual int Decode(char** vectorList, unsigned int numData, unsigned int erasureCount,
                       unsigned int* erasureLocs) = 0;
};  // end class NormDecoder

#endif  // _NORM_ENCODER
