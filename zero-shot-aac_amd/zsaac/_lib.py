"""ctypes binding of libzsaac_hip.so (the C-ABI declared in include/zsaac.h).

The library is built in-tree (``zero-shot-aac_amd/csrc/Makefile`` -> ``zsaac/libzsaac_hip.so``)
so it travels to the GPU box with the repo.  There is NO fallback: if the library is missing or
the device is not gfx950, every op raises — the product path never silently runs elsewhere.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# ZSAAC_LIB: another in-tree build of the same sources (A/B variants, e.g. libzsaac_hip_r4b.so)
LIB_PATH = (os.path.join(HERE, os.path.basename(os.environ["ZSAAC_LIB"]))
            if os.environ.get("ZSAAC_LIB") else os.path.join(HERE, "libzsaac_hip.so"))
CSRC = os.path.join(os.path.dirname(HERE), "csrc")

ZS_F32, ZS_BF16 = 0, 1
ACT_NONE, ACT_GELU_ERF, ACT_GELU_TANH, ACT_RELU, ACT_TANH = 0, 1, 2, 3, 4

P = C.c_void_p
I = C.c_int
F = C.c_float
L = C.c_long

# name -> argtypes (restype is always c_int).  Mirrors include/zsaac.h one-to-one; the CPU test
# suite checks this table against the header and the .so's dynamic symbols.
SIGNATURES = {
    "zs_version": [],
    "zs_last_error": [C.c_char_p, C.c_size_t],
    "zs_device_arch": [C.c_char_p, C.c_size_t],
    "zs_tune_set": [C.c_char_p, I],
    "zs_stream_create": [P, I],
    "zs_stream_create_masked": [P, P, I],
    "zs_stream_spin": [I, P],
    "zs_stream_destroy": [P],
    "zs_logmel": [P, I, I, P, P, P, P, P, P, P, P, P, P, P],
    "zs_wav2img": [P, I, I, P, P],
    "zs_pack_clips": [P, P, P, I, I, P, P],
    "zs_patch_embed": [P, I, P, P, P, P, P, P],
    "zs_layernorm": [P, I, I, I, P, P, P, F, P, I, I, P],
    "zs_gemm": [I, I, I, I, P, I, P, I, P, P, I, P, I, I, I, I, P, P],
    "zs_gemm_workspace_floats": [I, I, I],
    "zs_gemm_ln": [I, I, I, P, I, P, P, F, P, I, P, P, I, P, I, I, I, P],
    "zs_gemm_ln_f32": [I, I, I, P, I, P, P, F, P, I, P, P, I, P, I, I, P],
    "zs_l2norm_rows": [P, I, I, F, P, P],
    "zs_window_attention": [P, I, I, I, I, I, I, I, P, P, I, P],
    "zs_swin_block": [P, I, I, I, I, I, I, P, P, P, P, P, P, P, P, P, P, P, P, P, P],
    "zs_patch_merge_ln": [P, I, I, I, I, P, P, P, I, P],
    "zs_ln_meanpool": [P, I, I, I, P, P, P, P],
    "zs_conv3x3_bn_relu": [P, I, I, I, I, P, I, P, P, P, I, P],
    "zs_avgpool2": [P, I, I, I, I, P, I, P],
    "zs_cnn_head": [P, I, I, I, I, P, I, P],
    "zs_cast": [P, L, P, I, P],
    "zs_prompt_assemble": [P, I, I, P, I, I, P, P, I, P, I, P, P, P],
    "zs_row_attention": [P, I, P, P, I, I, I, P, I, I, I, F, P, I, I, P],
    "zs_row_attention_kv": [P, I, I, P, I, F, P, I, P, P, I, I, P],
    "zs_cross_attention": [P, I, P, P, I, I, I, I, I, I, F, P, I, I, P],
    "zs_label_topk": [P, I, I, P, I, I, P, P, P],
    "zs_gpt2_prefill_embed": [P, P, I, P, I, I, P, P, I, I, I, P, P, P, P, I, P],
    "zs_kv_write": [P, I, I, I, I, P, I, P, P, I, I, P],
    "zs_decode_attention": [P, I, I, I, P, P, I, P, P, P, I, P],
    "zs_embed_tokens": [P, P, P, P, I, I, P, I, P],
    "zs_embed_tokens_map": [P, P, P, I, P, P, I, I, P, P, I, P],
    "zs_decode_attention_map": [P, I, P, I, I, I, P, P, I, P, P, P, I, P],
    "zs_compact_rows": [P, I, P, P, P],
    "zs_greedy_step_map": [P, P, I, P, I, I, P, I, I, I, P, P, P, P, P, P, P],
    "zs_lmhead_topk": [I, I, I, I, P, I, P, I, I, P, P, P, P],
    "zs_lmhead_topk_t": [I, I, I, I, P, I, P, I, I, F, P, P, P, P],
    "zs_lmhead_nblk": [I],
    "zs_argmax_finalize": [P, P, I, I, P, P],
    "zs_prefix_ids_assemble": [P, I, P, P, I, I, I, P, P],
    "zs_greedy_step": [P, P, I, I, P, I, I, I, P, P, P, P, P, P, P],
    "zs_greedy_init": [I, P, P, P, P, P, I, P, P, P],
    "zs_decode_persist_workspace_bytes": [],
    "zs_gpt2_decode_persist": [I, I, I, I, I, I, P, P, P, F, P, P, P, P, P, P, P, P, P, P, P, L, I, I, P],
    "zs_gpt2_decode_phases": [I, I, I, I, I, I, P, P, P, F, P, P, P, P, P, P, P, P, P, P, P, L, I, I, P],
    "zs_decode_persist_f32_workspace_bytes": [],
    "zs_gpt2_decode_persist_f32": [I, I, I, I, I, I, P, P, P, F, P, P, P, P, P, P, P, P, P, P, P, L, I, I, P],
    "zs_gpt2_decode_phases_f32": [I, I, I, I, I, I, P, P, P, F, P, P, P, P, P, P, P, P, P, P, P, L, I, I, P],
    "zs_decode_persist_status": [P, P],
    "zs_decode_persist_set_stamps": [P, I, P],
    "zs_beam_step": [P, P, P, I, I, I, I, I, I, P, I, P, P, P, P, P, P, P, I, P, P, P, P],
    "zs_bert_embed_ln": [P, I, I, P, P, P, P, P, F, P, P, I, P],
    "zs_layernorm_dual": [P, I, I, I, P, P, F, P, I, P, I, I, P],
    "zs_row_topk": [P, I, I, L, I, I, P, P, P],
    "zs_magic_expand": [P, P, I, I, I, P, P, P],
    "zs_magic_maxcos": [P, I, I, P, I, P, P, P, I, P],
    "zs_magic_score": [P, P, P, P, I, I, I, I, I, F, F, F, P, P],
    "zs_fp8_gemm_rows": [P, I, P, P, I, I, I, P, L, I, P],
    "zs_fp8_splits": [I],
    "zs_fp8_gemm_run": [P, I, P, P, I, I, I, I, I, P, L, I, P, I, P, I, F, P],
    "zs_mistral_add_ss": [P, P, I, L, I, I, P, P, P],
    "zs_fp8_unpack_bf16": [P, I, I, P, P],
    "zs_scale_cols": [P, I, I, I, P, P],
    "zs_mistral_embed": [P, I, P, I, P, I, P, P, I, I, P, I, P],
    "zs_mistral_add_rmsnorm": [P, P, I, L, I, I, F, P, P, I, P],
    "zs_mistral_rope_kv": [P, I, L, I, I, I, P, I, P, P, P, P, P, I, I, P],
    "zs_mistral_silu_mul": [P, I, L, I, I, P, I, P],
    "zs_mistral_attention": [P, I, I, I, P, I, P, P, I, P, I, P],
    "zs_mistral_decode_attention": [P, I, L, I, I, I, P, P, P, P, P, I, P, I, P],
    "zs_magic_score_t": [P, P, P, P, I, I, I, I, I, F, F, F, F, P, P],
    "zs_magic_step": [P, P, I, I, I, I, I, I, I, P, P, P, P, P, I, P, I, P, P, P, P, P, I, P],
}

_lib = None
_lock = threading.Lock()


class ZsError(RuntimeError):
    pass


def build(force: bool = False, jobs: int = 8) -> str:
    """Compile libzsaac_hip.so for gfx950 with hipcc (cross-compiles without a GPU)."""
    cmd = ["make", "-C", CSRC, f"-j{jobs}"]
    if force:
        subprocess.run(["make", "-C", CSRC, "clean"], check=True, capture_output=True)
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise ZsError(f"building libzsaac_hip.so failed:\n{r.stdout}\n{r.stderr}")
    return LIB_PATH


def lib():
    """Load (once) and return the ctypes library; raises if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ZsError(f"{LIB_PATH} not found: run `make -C {CSRC}` "
                              "(or __graft_entry__.build()); there is no CPU fallback")
            h = C.CDLL(LIB_PATH)
            for name, args in SIGNATURES.items():
                fn = getattr(h, name)
                fn.argtypes = args
                fn.restype = C.c_int
            # experiment knobs for A/B runs, e.g. ZSAAC_TUNE="gemm_lean=0,fast_xcd=0"
            for kv in filter(None, os.environ.get("ZSAAC_TUNE", "").split(",")):
                k, v = kv.split("=")
                if h.zs_tune_set(k.strip().encode(), int(v)) != 0:
                    raise ZsError(f"ZSAAC_TUNE: unknown knob {k!r}")
            _lib = h
    return _lib


def last_error() -> str:
    buf = C.create_string_buffer(2048)
    lib().zs_last_error(buf, len(buf))
    return buf.value.decode(errors="replace")


def call(name: str, *args) -> int:
    rc = getattr(lib(), name)(*args)
    if rc < 0:
        raise ZsError(f"{name} failed ({rc}): {last_error()}")
    return rc


def device_arch() -> str:
    buf = C.create_string_buffer(256)
    call("zs_device_arch", buf, len(buf))
    return buf.value.decode()
