// nfecCodecBase.h -- the state every GPU-backed NORM codec class carries (one nfec codec
// handle plus the Init parameters), and the batch extensions beyond the reference surface.
//
// Included by normEncoderRS8.h, normEncoderRS16.h and normEncoderMDP.h of this directory.  The
// library (norm_amd/csrc/norm_codecs.cpp) and every NORM translation unit compile the codec
// classes from these same headers, so their layout is one definition everywhere.
#ifndef NFEC_CODEC_BASE_H
#define NFEC_CODEC_BASE_H

#include "normEncoder.h"
#include "../nfec.h"

class NfecCodecBase
{
  public:
    // GPU used by codecs created afterwards in this process; clears a device list set by
    // SetDevices (which spreads one codec over several GPUs from one process)
    static void SetDevice(int device) { default_device = device; num_devices = 0; devices_chosen = true; }
    static int GetDevice() { return default_device; }
    // Several GPUs for codecs created afterwards (at most kMaxDevices; a device may repeat):
    // Init creates one codec striped over them (nfec_codec_create_ex), so a single-process
    // caller -- one NORM session's encoder (normSession.cpp:834-889) -- spreads its host batches
    // over the node's GPUs in contiguous block ranges.  count <= 1 means SetDevice(devices[0]).
    enum { kMaxDevices = 64 };
    static bool SetDevices(const int* devices, int count);
    static int GetDevices(int* devices, int cap);  // the list (count returned; 1: the one device)
    // With no usable gfx950 device in the process (nfec_device_count() == 0) and no device
    // chosen by SetDevice / SetDevices, Init still succeeds when both per-call paths are on the
    // host (the defaults): the codec is host-only (NFEC_OPT_HOST_ONLY, a one-line notice on
    // stderr), Encode / Decode run on the CPU and the batch calls return NFEC_EDEVICE.  Any other
    // device failure (a bad ordinal or device list, an allocation failure on a present GPU) makes
    // Init fail, as does SetHostFallback(false).
    static void SetHostFallback(bool on) { host_fallback = on; }
    static bool GetHostFallback() { return host_fallback; }
    bool IsHostOnly() const;
    // Where Encode runs, the incremental sender's per-segment call (normObject.cpp:2038-2052):
    // on the host CPU (default; nfec_encode_segment_host, under a microsecond per 1.4 KB
    // segment) or as a GPU round trip (nfec_encode_segment, ~20-160 us).
    static void SetSegmentEncodeOnHost(bool on) { segment_on_host = on; }
    static bool GetSegmentEncodeOnHost() { return segment_on_host; }
    // Where a one-block Decode runs (NormSenderNode::Decode, normNode.h:484-487): on the host
    // CPU (default, nfec_decode_vectors_host) unless nfec_decode_host_preferred finds the repair
    // too large for it, else on the GPU (nfec_decode_vectors).  The batch calls always use the GPU.
    static void SetDecodeOnHost(bool on) { decode_on_host = on; }
    static bool GetDecodeOnHost() { return decode_on_host; }
    nfec_codec* Handle() const { return codec; }
    // Batched device-resident calls (see nfec_encode / nfec_decode): the throughput path for
    // block-at-once call sites such as NormObject::CalculateBlockParity (normObject.cpp:2203-2229).
    int EncodeBlocks(const nfec_block_batch* batch, void* stream);
    int DecodeBlocks(const nfec_block_batch* batch, const uint16_t* erasureLocs, uint32_t erasureStride,
                     const uint16_t* erasureCounts, int32_t* status, void* stream);

  protected:
    NfecCodecBase() : codec(0), ndata(0), npar(0), vector_size(0) {}
    ~NfecCodecBase() {}
    bool InitCodec(int kind, unsigned int numData, unsigned int numParity, UINT16 vectorSize);
    void DestroyCodec();
    nfec_codec* codec;
    unsigned int ndata;        // max data pkts per block (k)
    unsigned int npar;         // No. of parity packets (n-k)
    unsigned int vector_size;  // Size of biggest vector to encode
    static int default_device;
    static int device_list[kMaxDevices];
    static int num_devices;     // 0: default_device alone
    static bool segment_on_host;
    static bool decode_on_host;
    static bool host_fallback;
    static bool devices_chosen;  // SetDevice / SetDevices called: no host-only fallback
};

#endif  // NFEC_CODEC_BASE_H
