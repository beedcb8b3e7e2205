"""CPU: the host-side AddressSanitizer build (SURVEY §5 sanitizers).  csrc/Makefile's `asan`
target compiles every zs_* entry's host code (argument validators, plan selection, the C-ABI
glue) with -fsanitize=address, host only; tools/asan_abi.py then calls every entry of the binding
table with all-zero, negative and size-1 arguments under the ASan runtime.  Every call must
return without an ASan report, and with an error code (< 0) or 0 (an empty problem); the size
queries return their value.  (First build: ~2 min, the device code compiles as usual.)"""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "zero-shot-aac_amd", "csrc")
LIB = os.path.join(CSRC, "build_asan", "libzsaac_host_asan.so")
CLANG = "/opt/rocm/lib/llvm/bin/clang"


def test_host_validators_under_asan():
    if not os.path.exists(CLANG):
        pytest.skip("no ROCm clang")
    r = subprocess.run(["make", "-C", CSRC, "-j8", "asan"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
    rt = subprocess.run([CLANG, "-print-file-name=libclang_rt.asan-x86_64.so"],
                        capture_output=True, text=True).stdout.strip()
    assert os.path.exists(rt), rt
    env = dict(os.environ)
    # the ASan runtime must come first; anything already preloaded stays after it
    env["LD_PRELOAD"] = rt + (":" + env["LD_PRELOAD"] if env.get("LD_PRELOAD") else "")
    env["ASAN_OPTIONS"] = "detect_leaks=0:abort_on_error=0:exitcode=99"
    r = subprocess.run(["python3", os.path.join(ROOT, "tools", "asan_abi.py"), LIB], env=env,
                       capture_output=True, text=True, timeout=600)
    assert "ERROR: AddressSanitizer" not in r.stderr, r.stderr[-4000:]
    assert r.returncode == 0, (r.returncode, r.stderr[-4000:])
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["functions"] >= 60
    # size / count queries return their value; everything else an error code or 0
    queries = {"zs_decode_persist_workspace_bytes", "zs_decode_persist_f32_workspace_bytes", "zs_fp8_splits",
               "zs_last_error", "zs_lmhead_nblk", "zs_version", "zs_gemm_workspace_floats"}
    bad = {k: v for k, v in res["rc"].items() if k not in queries and any(c > 0 for c in v)}
    assert not bad, bad
