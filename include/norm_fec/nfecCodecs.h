// nfecCodecs.h -- all six GPU-backed NORM codec classes in one include.
//
// The classes are declared in the reference-named headers of this directory
// (normEncoderRS8.h, normEncoderRS16.h, normEncoderMDP.h; reference include/normEncoderRS8.h:7-66,
// normEncoderRS16.h:7-65, normEncoderMDP.h:38-84), which is what NORM's own sources include.
// This header is a convenience for code written against the engine directly.
#ifndef NFEC_CODECS_H
#define NFEC_CODECS_H

#include "normEncoderMDP.h"
#include "normEncoderRS8.h"
#include "normEncoderRS16.h"

#endif
