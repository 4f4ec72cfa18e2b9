"""Python mirror of NORM's FEC plugin surface, backed by the MI355X kernels.

Class names, method names, argument meaning and return values follow the reference
classes (include/normEncoder.h:38-54, normEncoderRS8.h, normEncoderRS16.h,
normEncoderMDP.h) so parity tests read like the reference's own fecTest
(src/common/fecTest.cpp):

    enc = NormEncoderRS8(); enc.Init(numData, numParity, vectorSize)
    enc.Encode(segmentId, dataVector, parityVectorList)      # parity ^= G[k+i][seg] * data
    dec = NormDecoderRS8(); dec.Init(numData, numParity, vectorSize)
    dec.Decode(vectorList, numData, erasureCount, erasureLocs) -> erasureCount | 0

On top of the per-call surface, `encode_blocks` / `decode_blocks` take a batch of blocks
resident in HBM (a torch uint8 CUDA tensor shaped [nblocks, k+m, seg_stride]) -- the
performance path.  Everything runs through libnfec.so; nothing here computes.  The per-call
Encode / Decode follow the C++ drop-in's defaults: the library's host CPU paths
(nfec_encode_segment_host, and nfec_decode_vectors_host unless the repair is very large), with
host=False for the GPU round trip.
"""
import ctypes

from . import _native as N


def _addr_ro(buf):
    """Address of a read-only byte buffer (bytes, bytearray, numpy array, memoryview)."""
    if hasattr(buf, "ctypes"):
        return buf.ctypes.data, buf
    if isinstance(buf, bytes):
        keep = ctypes.create_string_buffer(buf, len(buf))
        return ctypes.addressof(keep), keep
    mv = memoryview(buf)
    keep = (ctypes.c_char * mv.nbytes).from_buffer(mv)
    return ctypes.addressof(keep), keep


def _addr_rw(buf):
    if buf is None:
        return None, None
    if hasattr(buf, "ctypes"):
        return buf.ctypes.data, buf
    mv = memoryview(buf)
    keep = (ctypes.c_char * mv.nbytes).from_buffer(mv)
    return ctypes.addressof(keep), keep


def _stream_handle(stream):
    if stream is not None:
        return ctypes.c_void_p(int(getattr(stream, "cuda_stream", stream)))
    import torch

    return ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def _tensor_ptr(t, what):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError(f"{what} must be a CUDA (HIP) tensor")
    if not t.is_contiguous():
        raise ValueError(f"{what} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def device_count():
    return N.lib().nfec_device_count()


def build_generator(kind, num_data, num_parity):
    """Host-only generator parity rows (m x k) as a numpy array (no GPU needed)."""
    import numpy as np

    dtype = np.uint16 if kind == N.NFEC_RS16 else np.uint8
    out = np.zeros((num_parity, num_data), dtype)
    N.check(N.lib().nfec_build_generator(kind, num_data, num_parity, out.ctypes.data, out.nbytes),
            "nfec_build_generator")
    return out


class BlockLayout:
    """Contiguous HBM layout of a batch: block b, slot s at (b*(k+m) + s) * seg_stride."""

    def __init__(self, num_data, num_parity, vector_size, seg_stride=None):
        self.k, self.m, self.vec = num_data, num_parity, vector_size
        self.seg_stride = seg_stride or ((vector_size + 7) // 8 * 8)

    def empty(self, nblocks, device="cuda"):
        import torch

        return torch.zeros((nblocks, self.k + self.m, self.seg_stride), dtype=torch.uint8, device=device)


def _batch_struct(blocks, num_data, accumulate):
    if blocks.dtype.itemsize != 1 or blocks.dim() != 3:
        raise ValueError("blocks must be a uint8 tensor [nblocks, slots, seg_stride]")
    b = N.BlockBatch()
    b.blocks = blocks.data_ptr()
    b.block_stride = blocks.stride(0)
    b.seg_stride = blocks.stride(1)
    b.nblocks = blocks.shape[0]
    b.num_data = num_data.data_ptr() if num_data is not None else None
    b.flags = N.NFEC_ACCUMULATE if accumulate else 0
    if blocks.stride(2) != 1:
        raise ValueError("segment bytes must be contiguous")
    return b


class _Codec:
    """device: the GPU; devices: several GPUs (or one GPU listed several times) for one codec that
    stripes host batches over them (nfec_codec_create_ex); options: NFEC_OPT_* flags."""
    KIND = None

    def __init__(self, device=0, devices=None, options=0):
        self.device = device
        self.devices = list(devices) if devices else [device]
        self.options = options
        self._h = ctypes.c_void_p()
        self.ndata = self.npar = self.vector_size = 0

    # -- reference surface --
    def Init(self, numData, numParity, vectorSize):
        self.Destroy()
        cfg = N.CodecConfig()
        cfg.kind = self.KIND
        cfg.num_data, cfg.num_parity, cfg.vector_size = numData, numParity, vectorSize
        devs = (ctypes.c_int32 * len(self.devices))(*self.devices)
        cfg.devices = ctypes.cast(devs, ctypes.POINTER(ctypes.c_int32))
        cfg.num_devices = len(self.devices)
        cfg.flags = self.options
        rc = N.lib().nfec_codec_create_ex(ctypes.byref(cfg), ctypes.byref(self._h))
        if rc == N.NFEC_ERANGE:
            return False  # reference: PLOG(PL_FATAL) + return false (normEncoderRS8.cpp:405-409)
        N.check(rc, "nfec_codec_create")
        self.ndata, self.npar, self.vector_size = numData, numParity, vectorSize
        return True

    def Destroy(self):
        if self._h:
            N.lib().nfec_codec_destroy(self._h)
            self._h = ctypes.c_void_p()

    def __del__(self):
        try:
            self.Destroy()
        except Exception:
            pass

    def GetNumData(self):
        return self.ndata

    def GetNumParity(self):
        return self.npar

    def GetVectorSize(self):
        return self.vector_size

    def num_devices(self):
        """The device ordinals the codec runs on (nfec_codec_num_devices)."""
        self._need()
        n = N.check(N.lib().nfec_codec_num_devices(self._h, None, 0), "nfec_codec_num_devices")
        out = (ctypes.c_int32 * n)()
        N.lib().nfec_codec_num_devices(self._h, out, n)
        return list(out)

    def generator(self):
        import numpy as np

        dtype = np.uint16 if self.KIND == N.NFEC_RS16 else np.uint8
        out = np.zeros((self.npar, self.ndata), dtype)
        N.check(N.lib().nfec_codec_get_generator(self._h, out.ctypes.data, out.nbytes), "nfec_codec_get_generator")
        return out

    def features(self):
        """Bit mask of the encode paths the codec chose (NFEC_FEATURE_*, include/nfec.h)."""
        self._need()
        rc = N.lib().nfec_codec_features(self._h)
        N.check(min(rc, 0), "nfec_codec_features")
        return rc

    def encode_paths(self):
        """Device-batch encodes so far per path that took them, {name: count} (NFEC_PATH_*,
        include/nfec.h): which kernel family a batch shape reaches."""
        self._need()
        cnt = (ctypes.c_uint64 * N.NFEC_PATH_COUNT)()
        rc = N.lib().nfec_codec_encode_paths(self._h, cnt, N.NFEC_PATH_COUNT)
        N.check(min(rc, 0), "nfec_codec_encode_paths")
        return {name: int(cnt[i]) for i, name in enumerate(N.PATH_NAMES)}

    def decode_paths(self):
        """Device-batch decodes so far per path that took them, {name: count} (NFEC_DPATH_*)."""
        self._need()
        cnt = (ctypes.c_uint64 * N.NFEC_DPATH_COUNT)()
        rc = N.lib().nfec_codec_decode_paths(self._h, cnt, N.NFEC_DPATH_COUNT)
        N.check(min(rc, 0), "nfec_codec_decode_paths")
        return {name: int(cnt[i]) for i, name in enumerate(N.DPATH_NAMES)}

    def _need(self):
        if not self._h:
            raise RuntimeError("codec not initialised (call Init)")


class _Encoder(_Codec):
    def Encode(self, segmentId, dataVector, parityVectorList, host=True):
        """NormEncoder::Encode.  host=True (the drop-in's default): nfec_encode_segment_host, the
        product on the calling CPU; host=False: the GPU round trip, nfec_encode_segment."""
        self._need()
        daddr, dkeep = _addr_ro(dataVector)
        keeps = []
        arr = (ctypes.c_void_p * self.npar)()
        for i in range(self.npar):
            a, k = _addr_rw(parityVectorList[i])
            arr[i] = a
            keeps.append(k)
        fn = "nfec_encode_segment_host" if host else "nfec_encode_segment"
        N.check(getattr(N.lib(), fn)(self._h, segmentId, daddr, arr), fn)

    def encode_blocks(self, blocks, num_data=None, accumulate=False, stream=None):
        """Parity for every block of a device batch (slots [nd, nd+m) of each block)."""
        self._need()
        b = _batch_struct(blocks, num_data, accumulate)
        N.check(N.lib().nfec_encode(self._h, ctypes.byref(b), _stream_handle(stream)), "nfec_encode")

    def encode_blocks_host(self, blocks, num_data=None, accumulate=False):
        """Same as encode_blocks for a numpy uint8 array [nblocks, slots, seg_stride] in host memory."""
        self._need()
        b = N.BlockBatch()
        b.blocks = blocks.ctypes.data
        b.block_stride = blocks.strides[0]
        b.seg_stride = blocks.strides[1]
        b.nblocks = blocks.shape[0]
        b.num_data = num_data.ctypes.data if num_data is not None else None
        b.flags = N.NFEC_ACCUMULATE if accumulate else 0
        N.check(N.lib().nfec_encode_host(self._h, ctypes.byref(b)), "nfec_encode_host")


    def encode_vectors_host(self, vectors, num_data=None, accumulate=False):
        """Batch form of CalculateBlockParity on NORM-style segment lists: vectors is a list of
        blocks, each a list of k+m (or numData_b+m) writable host buffers (numpy uint8 arrays or
        anything with a buffer) -- slots [0, numData_b) source, then m parity."""
        self._need()
        arr, keep, nd = _vector_table(vectors, self.ndata + self.npar, num_data, self.ndata)
        N.check(N.lib().nfec_encode_host_vectors(self._h, arr, len(vectors), nd,
                                                 N.NFEC_ACCUMULATE if accumulate else 0), "nfec_encode_host_vectors")


    def encode_vectors_host_async(self, vectors, num_data=None, accumulate=False):
        """encode_vectors_host queued on the codec's worker thread; returns a Request."""
        self._need()
        arr, keep, nd = _vector_table(vectors, self.ndata + self.npar, num_data, self.ndata)
        h = ctypes.c_void_p()
        N.check(N.lib().nfec_encode_host_vectors_async(self._h, arr, len(vectors), nd,
                                                       N.NFEC_ACCUMULATE if accumulate else 0, ctypes.byref(h)),
                "nfec_encode_host_vectors_async")
        return Request(h, (arr, keep, vectors, self), None)


class _Decoder(_Codec):
    def Decode(self, vectorList, numData, erasureCount, erasureLocs, host=None):
        """NormDecoder::Decode on one block.  host: None -- the drop-in's choice
        (nfec_decode_host_preferred: the host CPU for RS8 and small RS16, else the GPU);
        True / False -- force nfec_decode_vectors_host / nfec_decode_vectors."""
        self._need()
        n = numData + self.npar
        arr = (ctypes.c_void_p * n)()
        keeps = []
        for i in range(n):
            a, k = _addr_rw(vectorList[i])
            arr[i] = a
            keeps.append(k)
        locs = (ctypes.c_uint32 * max(1, erasureCount))(*list(erasureLocs)[:erasureCount])
        if host is None:
            host = N.lib().nfec_decode_host_preferred(self._h, numData, erasureCount) == 1
        if host:
            return N.check(N.lib().nfec_decode_vectors_host(self._h, arr, numData, erasureCount, locs),
                           "nfec_decode_vectors_host")
        rc = N.lib().nfec_decode_vectors(self._h, arr, numData, erasureCount, locs)
        return N.check(rc, "nfec_decode_vectors")

    def decode_blocks(self, blocks, erasure_locs, erasure_counts, num_data=None, status=None, accumulate=False,
                      stream=None):
        """Repair every block of a device batch.  erasure_locs: int16/uint16 [nblocks, stride]
        sorted slot indices; erasure_counts: int16/uint16 [nblocks]; returns int32 status
        [nblocks] (reference Decode return value per block)."""
        import torch

        self._need()
        if status is None:
            status = torch.empty(blocks.shape[0], dtype=torch.int32, device=blocks.device)
        b = _batch_struct(blocks, num_data, accumulate)
        rc = N.lib().nfec_decode(self._h, ctypes.byref(b), _tensor_ptr(erasure_locs, "erasure_locs"),
                                 erasure_locs.shape[1], _tensor_ptr(erasure_counts, "erasure_counts"),
                                 _tensor_ptr(status, "status"), _stream_handle(stream))
        N.check(rc, "nfec_decode")
        return status

    def decode_blocks_host(self, blocks, erasure_locs, erasure_counts, num_data=None, accumulate=False):
        import numpy as np

        self._need()
        status = np.zeros(blocks.shape[0], np.int32)
        b = N.BlockBatch()
        b.blocks = blocks.ctypes.data
        b.block_stride = blocks.strides[0]
        b.seg_stride = blocks.strides[1]
        b.nblocks = blocks.shape[0]
        b.num_data = num_data.ctypes.data if num_data is not None else None
        b.flags = N.NFEC_ACCUMULATE if accumulate else 0
        N.check(N.lib().nfec_decode_host(self._h, ctypes.byref(b), erasure_locs.ctypes.data, erasure_locs.shape[1],
                                         erasure_counts.ctypes.data, status.ctypes.data), "nfec_decode_host")
        return status


    def decode_vectors_host_async(self, vectors, erasure_locs, erasure_counts, num_data=None, accumulate=False):
        """decode_vectors_host queued on the codec's worker thread: returns a Request at once
        (the receiver keeps going; Request.wait() gives the status array)."""
        import numpy as np

        self._need()
        arr, keep, nd = _vector_table(vectors, self.ndata + self.npar, num_data, self.ndata)
        locs = np.ascontiguousarray(erasure_locs, dtype=np.uint16)
        counts = np.ascontiguousarray(erasure_counts, dtype=np.uint16)
        status = np.zeros(len(vectors), np.int32)
        h = ctypes.c_void_p()
        N.check(N.lib().nfec_decode_host_vectors_async(self._h, arr, len(vectors), nd, locs.ctypes.data, locs.shape[1],
                                                       counts.ctypes.data, status.ctypes.data,
                                                       N.NFEC_ACCUMULATE if accumulate else 0, ctypes.byref(h)),
                "nfec_decode_host_vectors_async")
        return Request(h, (arr, keep, locs, counts, vectors, self), status)

    def decode_vectors_host(self, vectors, erasure_locs, erasure_counts, num_data=None, accumulate=False):
        """Receiver repair of many blocks given as NORM-style segment lists (None allowed for
        missing parity).  erasure_locs: uint16 [nblocks, stride]; erasure_counts: uint16
        [nblocks].  Returns int32 status [nblocks]."""
        import numpy as np

        self._need()
        arr, keep, nd = _vector_table(vectors, self.ndata + self.npar, num_data, self.ndata)
        locs = np.ascontiguousarray(erasure_locs, dtype=np.uint16)
        counts = np.ascontiguousarray(erasure_counts, dtype=np.uint16)
        status = np.zeros(len(vectors), np.int32)
        N.check(N.lib().nfec_decode_host_vectors(self._h, arr, len(vectors), nd, locs.ctypes.data, locs.shape[1],
                                                 counts.ctypes.data, status.ctypes.data,
                                                 N.NFEC_ACCUMULATE if accumulate else 0), "nfec_decode_host_vectors")
        return status


class Request:
    """An asynchronous segment-list batch (nfec_*_host_vectors_async).  Keeps the caller's
    buffers alive until completion; test() polls, wait() blocks and returns the status array
    (decode) or None (encode), raising NfecError if the call failed."""

    def __init__(self, handle, keep, status):
        self._h, self._keep, self._status = handle, keep, status

    def test(self):
        if not self._h:
            return True
        return N.check(N.lib().nfec_request_test(self._h), "nfec_request_test") == 1

    def wait(self):
        if self._h:
            h, self._h = self._h, None
            N.check(N.lib().nfec_request_wait(h), "nfec_request_wait")
            self._keep = None
        return self._status

    def __del__(self):
        try:
            self.wait()
        except Exception:
            pass


def _vector_table(vectors, n, num_data, k):
    """(void*[nblocks * n] pointer table, keep-alive list, num_data pointer or None)"""
    import numpy as np

    arr = (ctypes.c_void_p * (len(vectors) * n))()
    keep = []
    for b, blk in enumerate(vectors):
        for s, v in enumerate(blk):
            if v is None:
                continue
            a, kk = _addr_rw(v)
            arr[b * n + s] = a
            keep.append(kk)
    nd = None
    if num_data is not None:
        nd_arr = np.ascontiguousarray(num_data, dtype=np.uint16)
        keep.append(nd_arr)
        nd = nd_arr.ctypes.data
    return arr, keep, nd


class NormEncoderRS8(_Encoder):
    KIND = N.NFEC_RS8


class NormDecoderRS8(_Decoder):
    KIND = N.NFEC_RS8


class NormEncoderRS16(_Encoder):
    KIND = N.NFEC_RS16


class NormDecoderRS16(_Decoder):
    KIND = N.NFEC_RS16


class NormEncoderMDP(_Encoder):
    KIND = N.NFEC_MDP


class NormDecoderMDP(_Decoder):
    KIND = N.NFEC_MDP


# -- synthetic workload helpers (device kernels) --
def fill_blocks(blocks, num_data, vector_size, seed, first_block=0, per_block_num_data=None, stream=None):
    b = _batch_struct(blocks, per_block_num_data, False)
    N.check(N.lib().nfec_util_fill(ctypes.byref(b), num_data, vector_size, seed, first_block, _stream_handle(stream)),
            "nfec_util_fill")


def stream_copy(dst, src, stream=None):
    """dst[:] = src through the streaming copy kernel (bench's achievable-HBM figure)."""
    if dst.numel() * dst.element_size() != src.numel() * src.element_size():
        raise ValueError("stream_copy: size mismatch")
    N.check(N.lib().nfec_util_stream_copy(ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(src.data_ptr()),
                                          src.numel() * src.element_size(), _stream_handle(stream)),
            "nfec_util_stream_copy")


def make_erasures(nblocks, range_, count, seed, stride, first_block=0, device="cuda", stream=None):
    import torch

    locs = torch.zeros((nblocks, stride), dtype=torch.int16, device=device)
    counts = torch.zeros(nblocks, dtype=torch.int16, device=device)
    N.check(N.lib().nfec_util_erasures(ctypes.c_void_p(locs.data_ptr()), stride, ctypes.c_void_p(counts.data_ptr()),
                                       nblocks, range_, count, seed, first_block, _stream_handle(stream)),
            "nfec_util_erasures")
    return locs, counts


def zero_erasures(blocks, erasure_locs, erasure_counts, vector_size, stream=None):
    b = _batch_struct(blocks, None, False)
    N.check(N.lib().nfec_util_zero_slots(ctypes.byref(b), _tensor_ptr(erasure_locs, "erasure_locs"),
                                         erasure_locs.shape[1], _tensor_ptr(erasure_counts, "erasure_counts"),
                                         vector_size, _stream_handle(stream)), "nfec_util_zero_slots")
