"""npc -- NORM's offline file precoder (reference src/common/normPrecode.cpp) on the GPU path.

    python -m norm_amd.npc {encode|decode} input <inFile> [output <outFile>]
           [segment <segmentSize>][block numData][parity numParity]
           [auto <parityPercentage>][bmax <n>][imax <n>][ibuffer <n>][device <n>[,<n>...]]

The command language is the reference's (NormPrecodeApp::ProcessCommands / CommandType,
normPrecode.cpp:124-346): commands match by unambiguous prefix, "block" turns auto sizing
off, and with neither "block" nor "auto" the reference's default auto mode (100.0, i.e.
100x parity) applies.  Encoding writes <base name with '.' -> '_'>.npc in the current
directory unless "output" is given (:590-606); decoding writes to the name stored in the
file's meta segment unless "output" is given (:1142-1154).  "ibuffer" only chooses the
reference's I/O strategy, not the output, and is accepted and ignored.

The FEC encode/decode and the per-segment CRC-32 run on the GPU (libnfec.so,
nfec_npc_encode_file / nfec_npc_decode_file).
"""
import ctypes
import os
import sys

from . import _native as N


def default_params():
    p = N.NpcParams()
    N.lib().nfec_npc_default_params(ctypes.byref(p))
    return p


def make_params(segment=None, block=None, parity=None, auto=None, bmax=None, imax=None):
    """Parameters as the reference's command handlers set them (OnCommand, :152-300)."""
    p = default_params()
    if segment is not None:
        p.segment_size = int(segment)
    if block is not None:
        p.num_data = int(block)
        p.parity_fraction = -1.0
    if parity is not None:
        p.num_parity = int(parity)
    if auto is not None:
        if auto < 0:
            raise ValueError("npc: invalid block <auto> value")
        p.parity_fraction = float(auto) / 100.0
    if bmax is not None:
        p.b_max = int(bmax) if int(bmax) > 0 else 65536
    if imax is not None:
        p.i_max = max(0, int(imax))
    return p


def layout(params, file_size, encode=True):
    lay = N.NpcLayout()
    N.check(N.lib().nfec_npc_layout_for(ctypes.byref(params), file_size, 1 if encode else 0, ctypes.byref(lay)),
            "nfec_npc_layout_for")
    return lay


def positions(lay, first=0, count=None):
    import numpy as np

    count = lay.num_segments - first if count is None else count
    out = np.zeros(count, np.uint64)
    N.check(N.lib().nfec_npc_positions(ctypes.byref(lay), first, count, out.ctypes.data), "nfec_npc_positions")
    return out


def default_output_name(in_path):
    """<base name, last '.' -> '_'>.npc (NormPrecodeApp::Encode, :590-602)."""
    name = os.path.basename(in_path)
    dot = name.rfind(".")
    if dot >= 0:
        name = name[:dot] + "_" + name[dot + 1:]
    return name + ".npc"


def _device_list(device, devices):
    devs = [int(device)] if devices is None else [int(d) for d in devices]
    arr = (ctypes.c_int32 * max(1, len(devs)))(*devs)
    return arr, len(devs)


def encode_file(in_path, out_path=None, params=None, device=0, devices=None):
    """devices: a list of GPUs sharing the pass (contiguous block ranges), else `device` alone"""
    params = params or default_params()
    out_path = out_path or default_output_name(in_path)
    arr, n = _device_list(device, devices)
    N.check(N.lib().nfec_npc_encode_file_multi(ctypes.addressof(arr), n, os.fsencode(in_path), os.fsencode(out_path),
                                               ctypes.byref(params)),
            "nfec_npc_encode_file_multi")
    return out_path


def decode_file(in_path, out_path=None, params=None, device=0, devices=None):
    """-> (output path, bytes written)."""
    params = params or default_params()
    nbytes = ctypes.c_uint64()
    name = ctypes.create_string_buffer(4096)
    arr, n = _device_list(device, devices)
    N.check(N.lib().nfec_npc_decode_file_multi(ctypes.addressof(arr), n, os.fsencode(in_path),
                                               os.fsencode(out_path) if out_path else None,
                                               ctypes.byref(params), ctypes.byref(nbytes), name, len(name)),
            "nfec_npc_decode_file_multi")
    return (out_path or name.value.decode(errors="surrogateescape")), nbytes.value


# ---- command line (normPrecode.cpp:124-346) ----
_CMDS = ["-help", "+debug", "-encode", "-decode", "+input", "+output", "+segment", "+block", "+parity", "+auto",
         "+bmax", "+imax", "+ibuffer", "-background", "+device"]


def _command_type(cmd):
    """Unambiguous prefix match (CommandType, :318-346): '+' takes an argument."""
    hits = [c for c in _CMDS if c[1:].startswith(cmd)]
    if len(hits) != 1 or not cmd:
        return None, None
    return hits[0][1:], hits[0][0] == "+"


def _usage():
    sys.stderr.write("Usage:  npc {encode|decode} input <inFile> [output <outFile>]\n"
                     "            [segment <segmentSize>][block numData][parity numParity]\n"
                     "            [auto <parityPercentage>][bmax <n>][imax <n>][device <n>[,<n>...]]\n")


def main(argv=None):
    argv = list(sys.argv[1:] if argv is None else argv)
    encode, inp, outp, dev = True, None, None, [0]
    kw = {}
    i = 0
    while i < len(argv):
        name, takes = _command_type(argv[i])
        if name is None:
            sys.stderr.write(f"npc: error: Invalid command:{argv[i]}\n")
            return 1
        val = None
        if takes:
            if i + 1 >= len(argv):
                sys.stderr.write(f"npc: {name} missing argument\n")
                return 1
            val = argv[i + 1]
        i += 2 if takes else 1
        if name == "help":
            _usage()
            return 1
        if name in ("encode", "decode"):
            encode = name == "encode"
        elif name == "input":
            if not os.path.isfile(val):
                sys.stderr.write(f"npc: error opening input file: {val}\n")
                return 1
            inp = val
        elif name == "output":
            outp = val
        elif name == "segment":
            kw["segment"] = int(val)
        elif name == "block":
            kw["block"] = int(val)
        elif name == "parity":
            kw["parity"] = int(val)
        elif name == "auto":
            kw["auto"] = float(val)
        elif name == "bmax":
            kw["bmax"] = int(val)
        elif name == "imax":
            kw["imax"] = int(val)
        elif name == "device":
            dev = [int(d) for d in val.split(",")]  # a list shares the pass over those GPUs
        # debug, ibuffer, background: no effect on the output
    if inp is None:
        sys.stderr.write("npc: error: no input file given\n")
        _usage()
        return 1
    try:
        params = make_params(**kw)
        if encode:
            encode_file(inp, outp, params, devices=dev)
        else:
            decode_file(inp, outp, params, devices=dev)
    except (N.NfecError, ValueError) as e:
        sys.stderr.write(f"npc: {e}\n")
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
