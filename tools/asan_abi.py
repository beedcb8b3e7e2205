#!/usr/bin/env python3
"""Drives every zs_* entry of the host-only ASan build (csrc/Makefile `asan`) through its argument
validators with bad arguments, under the ASan runtime (tests/test_asan.py starts this with
LD_PRELOAD=libclang_rt.asan): all-zero arguments, negative sizes with null pointers, and size 1
with zero-filled host buffers (pointer tables read as null pointers).  Every call must return
(an error code, or 0 for an empty problem) without an ASan report; no GPU is touched (the host-only
build has no device code objects; a call that got past its validators would fail at the HIP
launch, which this host does not have).

    LD_PRELOAD=<asan rt> python3 tools/asan_abi.py <libzsaac_host_asan.so>
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "zero-shot-aac_amd"))

from zsaac._lib import SIGNATURES, F, I, L, P  # noqa: E402

# calls that need a device to be meaningful at all and never validate host memory
SKIP = {"zs_stream_create", "zs_stream_destroy", "zs_device_arch"}


def main(path):
    lib = C.CDLL(path)
    buf = C.create_string_buffer(1 << 16)            # zero-filled host memory
    bufp = C.cast(buf, C.c_void_p).value
    res = {}
    for name, sig in sorted(SIGNATURES.items()):
        if name in SKIP or not hasattr(lib, name):
            continue
        fn = getattr(lib, name)
        fn.restype = C.c_int
        argt = []
        for t in sig:
            argt.append({I: C.c_int, L: C.c_long, F: C.c_float, P: C.c_void_p}.get(t, t))
        fn.argtypes = argt
        out = []
        for mode in ("zero", "neg", "one_buf"):
            args = []
            for t in argt:
                if t is C.c_char_p:
                    args.append(None if mode != "one_buf" else b"x")
                elif t is C.c_void_p or (isinstance(t, type) and issubclass(t, C._Pointer)):
                    args.append(None if mode != "one_buf" else C.cast(bufp, t) if t is not C.c_void_p else bufp)
                elif t in (C.c_float, C.c_double):
                    args.append({"zero": 0.0, "neg": -1.0, "one_buf": 1.0}[mode])
                elif t in (C.c_size_t, C.c_uint, C.c_ulong):
                    args.append({"zero": 0, "neg": 0, "one_buf": 1}[mode])
                else:
                    args.append({"zero": 0, "neg": -1, "one_buf": 1}[mode])
            try:
                out.append(int(fn(*args)))
            except C.ArgumentError as e:
                raise SystemExit(f"{name} {mode}: {e} (argtypes {argt})")
        res[name] = out
    print(json.dumps({"calls": 3 * len(res), "functions": len(res), "rc": res}))


if __name__ == "__main__":
    main(sys.argv[1])
