// normEncoder.h -- NormEncoder / NormDecoder plugin surface for the MI355X FEC engine.
//
// Same abstract interface as the reference (include/normEncoder.h:38-54): a NORM engine
// built against this header (or against its own normEncoder.h, which declares the same
// classes) can construct the GPU-backed codecs below in place of the CPU ones at
// src/common/normSession.cpp:842-883 and src/common/normNode.cpp:295-357.
#ifndef NFEC_NORM_ENCODER_H
#define NFEC_NORM_ENCODER_H

#ifdef NFEC_WITH_PROTOLIB
#include "protokit.h"  // inside a NORM tree: protolib supplies UINT8/UINT16/UINT32
#else
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
};

class NormDecoder
{
  public:
    virtual ~NormDecoder();
    virtual bool Init(unsigned int numData, unsigned int numParity, UINT16 vectorSize) = 0;
    virtual void Destroy() = 0;
    virtual int Decode(char** vectorList, unsigned int numData, unsigned int erasureCount,
                       unsigned int* erasureLocs) = 0;
};

#endif
