"""Real-data evaluation harness: the reference's ``predict_prompt.py`` driver on the HIP pipeline.

Mirrors predict_prompt.py ``main`` (183-231) and ``make_preds`` (104-181) for the captioning
modes on the hot path (greedy ``generate2`` and ``generate_beam(beam_size=3)``):

* ``<test_dir>/params.json`` -> the model configuration (predict_prompt.py:193-196, 209-216);
* ``<test_dir>/best.pth`` -> the ClapCaption_prompt state dict (:220), loaded weights-only;
* ``--test_data`` pickle -> clips ``{"audio_embedding", "caption", "audio_id"}``
  (dataset/dataset.py:443-453, 477-479), loaded through the allow-list unpickler;
* ``params.sound_effect`` pickle -> the AudioSet label table (dataset/dataset.py:465-474);
* per clip: label top-k -> hard prompt -> clap_to_gpt -> get_prefix_tokens + generate2 /
  generate_beam, batched on the GPU (``CaptionPipeline``);
* ``<test_dir>/output.txt``: ``{"predictions": [{"filename", "caption", "prefix"}]}``
  (:172-181); ``scores.txt`` (:155-170) only when ``pycocoevalcap`` is importable (it is not in
  this image, and its SPICE/METEOR scorers need Java).

The tokenizer is GPT-2 byte-level BPE from a local ``vocab.json`` + ``merges.txt``
(``--tokenizer``; ``zsaac.bpe``).  ``--magic`` (predict_prompt.py:121-140) runs CLAP-guided
beam decoding, ``generate_beam_magic(beam_size=3, magic_width, alpha 0.1, beta 0.2)`` with
``audio_embeds = prefix``, batched on zsaac.magic.MagicDecoder; the CLAP checkpoint
(``--clap``, the reference's HTSAT-BERT-ZS.pt: ``{"model": ASE state dict}``) supplies the BERT
text tower and ``--bert_vocab`` its WordPiece vocabulary (bert-base-uncased's vocab.txt).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import safeload
from .bpe import GPT2BPE
from .pipeline import CaptionConfig, CaptionPipeline
from .tokenizer import TEMPLATE_IDS

# predict_prompt.py:19-22: applied over params.json (args.__dict__.update(params), line 197)
MAGIC_PARAMS = {"beta": 0.2, "alpha": 0.1}


def magic_settings(params: dict):
    """(magic_width, alpha, beta) as predict_prompt.py --magic uses them: magic_width from
    params.json (line 140), alpha / beta from the module-level params that overwrite it (197)."""
    return int(params.get("magic_width", 25)), MAGIC_PARAMS["alpha"], MAGIC_PARAMS["beta"]


def post_processing(captions) -> List[str]:
    """predict_prompt.py:83-92: append '.' when missing, lower-case."""
    out = []
    for item in captions:
        c = item["caption"] if isinstance(item, dict) else str(item)
        if c[-1] != ".":
            c = c + "."
        out.append(str(c.lower()))
    return out


def load_params(test_dir: str) -> Dict:
    with open(os.path.join(test_dir, "params.json"), "r") as f:
        return json.load(f)


def load_labels(path: str) -> Tuple[List[str], torch.Tensor]:
    """audioset_label.pkl -> (label strings, label embeddings [L, 1024]) in file order."""
    items = safeload.load_pickle(path)
    names = [str(it["label"]) for it in items]
    table = safeload.stack_rows([it["label_embedding"] for it in items])
    return names, table


def check_template(tokenizer) -> None:
    """The prompt kernel writes GPT-2's template ids ("There", " are", " something", " in",
    " this", " audio", ".", ","): the tokenizer must agree."""
    for piece, ids in TEMPLATE_IDS.items():
        got = tokenizer.encode(piece)
        if list(got) != list(ids):
            raise ValueError(f"tokenizer encodes {piece!r} as {got}, the prompt template uses {ids}")


def label_token_table(tokenizer, names: Sequence[str]) -> List[List[int]]:
    """Per label the ids of ``' ' + label.lower()`` (utils.py:164-174 lower-cases the chosen
    labels).  The device assembles a prompt from these per-piece ids, which equals encoding the
    whole prompt string only when the label ends on a pre-tokenizer boundary: checked here for
    the separators that can follow a label ("," and " in")."""
    out, bad = [], []
    comma, tail = tokenizer.encode(","), tokenizer.encode(" in")
    for n in names:
        s = " " + n.lower()
        ids = list(tokenizer.encode(s))
        if (list(tokenizer.encode(s + ",")) != ids + list(comma)
                or list(tokenizer.encode(s + " in")) != ids + list(tail)):
            bad.append(n)
        out.append(ids)
    if bad:
        raise ValueError(f"labels whose BPE merges across the separator (not supported by the "
                         f"device prompt assembly): {bad[:5]}{'...' if len(bad) > 5 else ''}")
    return out


def config_from_params(params: Dict, isbeam: bool, dtype: torch.dtype, batch: int) -> CaptionConfig:
    """predict_prompt.py:209-216 ClapCaption_prompt arguments -> CaptionConfig."""
    if not params.get("is_rn", True):
        raise NotImplementedError("prefix_size 512 (is_rn false): the hot path is the 1024-d CLAP")
    if params.get("only_soft_prompt", False):
        raise NotImplementedError("only_soft_prompt: the hot path uses the hard prompt")
    mt = {"mlp": "mlp", "transformer": "transformer"}[params["mapping_type"]]
    return CaptionConfig(
        mapping_type=mt, dtype=dtype, batch=batch, beam=3 if isbeam else 0,
        sound_effect_num=int(params.get("sound_effect_num", 3)),
        normalize_prefix=bool(params.get("normalize_prefix", False)),
        prefix_length=int(params.get("prefix_length", 10)),
        clip_length=int(params.get("prefix_length_clip", 10)),
        mapper_layers=int(params.get("num_layers", 8)),
        prefix_tokens=True, use_graph=True)


def build_pipeline(test_dir: str, params: Dict, tokenizer, isbeam: bool = False,
                   dtype: torch.dtype = torch.float32, batch: int = 64,
                   device="cuda") -> Tuple[CaptionPipeline, List[str]]:
    check_template(tokenizer)
    names, table = load_labels(params["sound_effect"])
    ltok = label_token_table(tokenizer, names)
    sd = safeload.load_state_dict(os.path.join(test_dir, "best.pth"))
    cfg = config_from_params(params, isbeam, dtype, batch)
    return CaptionPipeline(sd, None, table, ltok, cfg, device=device), names


def make_preds(pipe: CaptionPipeline, tokenizer, all_data: List[Dict],
               ) -> Tuple[Dict[str, List[str]], Dict[str, List[str]], Dict[str, List[str]]]:
    """predict_prompt.py:104-153 over batches of ``pipe.cfg.batch`` clips: returns key2pred
    (lower-cased captions), key2pred_prefix (get_prefix_tokens strings) and key2refs."""
    key2refs: Dict[str, List[str]] = {}
    for it in all_data:
        key2refs[it["audio_id"]] = post_processing(it.get("caption", []))
    key2pred: Dict[str, List[str]] = {}
    key2pred_prefix: Dict[str, List[str]] = {}
    B = pipe.cfg.batch
    for c0 in range(0, len(all_data), B):
        chunk = all_data[c0:c0 + B]
        emb = safeload.stack_rows([it["audio_embedding"] for it in chunk]).to(pipe.dev)
        out = pipe.caption_emb(emb)
        caps = out.captions()                    # greedy: generated ids; beam: best beam
        prefs = out.prefix_token_lists()
        for it, ids, pids in zip(chunk, caps, prefs):
            key2pred[it["audio_id"]] = [tokenizer.decode(ids).lower()]
            key2pred_prefix[it["audio_id"]] = [tokenizer.decode(pids)]
    return key2pred, key2pred_prefix, key2refs


def make_preds_magic(pipe: CaptionPipeline, tokenizer, all_data: List[Dict], clap_sd, bert_tok,
                     width: int = 25, alpha: float = 0.1, beta: float = 0.2, beam: int = 3,
                     entry_length: int = 20):
    """predict_prompt.py:121-140 with ``--magic``: per clip generate_beam_magic(model, clap,
    tokenizer, audio_embeds=prefix, embed=prefix_embed, beam_size=3, alpha, beta, magic_width)[0]
    (entry_length 20, the function's default), batched over ``pipe.cfg.batch`` clips."""
    from . import ops
    from .bert import BertTextEngine
    from .magic import MagicDecoder
    key2refs: Dict[str, List[str]] = {it["audio_id"]: post_processing(it.get("caption", []))
                                      for it in all_data}
    key2pred: Dict[str, List[str]] = {}
    key2pred_prefix: Dict[str, List[str]] = {}
    B = pipe.cfg.batch
    bert = BertTextEngine(clap_sd, pipe.dev, pipe.cfg.dtype, max_texts=B * beam * width)
    mag = MagicDecoder(pipe.gpt, bert, B, pipe.Pmax, beam=beam, width=width, max_steps=entry_length)
    for c0 in range(0, len(all_data), B):
        chunk = all_data[c0:c0 + B]
        emb = safeload.stack_rows([it["audio_embedding"] for it in chunk]).to(pipe.dev)
        n = emb.shape[0]
        pipe.begin_emb(emb)                      # prompt, mapper, get_prefix_tokens (+ prefill)
        prefs = pipe.result().prefix_token_lists()
        prefix = pipe.prefix[:n]
        soft = pipe.mapper(prefix)
        res = mag.beam_magic(pipe.hard_ids[:n], pipe.hard_len[:n], soft, pipe.cfg.prefix_length,
                             prefix, tokenizer, bert_tok, beam, width, entry_length, alpha, beta,
                             soft_ld=pipe.mapper.soft_ld)
        for it, (toks, _), pids in zip(chunk, res, prefs):
            key2pred[it["audio_id"]] = [tokenizer.decode(toks[0]).lower()]
            key2pred_prefix[it["audio_id"]] = [tokenizer.decode(pids)]
    return key2pred, key2pred_prefix, key2refs


def write_outputs(test_dir: str, key2pred, key2pred_prefix, key2refs) -> Optional[Dict]:
    """output.txt exactly as predict_prompt.py:172-181; scores.txt (:155-170) when the
    captioning metrics are importable."""
    pred_data = [{"filename": k, "caption": "".join(p[0]), "prefix": "".join(key2pred_prefix[k][0])}
                 for k, p in key2pred.items()]
    with open(os.path.join(test_dir, "output.txt"), "w") as f:
        json.dump({"predictions": pred_data}, f, indent=4)
    try:
        from pycocoevalcap.bleu.bleu import Bleu          # noqa: F401
    except ImportError:
        print("pycocoevalcap not importable: scores.txt not written", file=sys.stderr)
        return None
    from pycocoevalcap.bleu.bleu import Bleu
    from pycocoevalcap.cider.cider import Cider
    from pycocoevalcap.meteor.meteor import Meteor
    from pycocoevalcap.rouge.rouge import Rouge
    from pycocoevalcap.spice.spice import Spice
    from pycocoevalcap.tokenizer.ptbtokenizer import PTBTokenizer
    tok = PTBTokenizer()

    def fmt(d):
        return {k: [{"audio_id": k, "id": i, "caption": c} for i, c in enumerate(v)] for k, v in d.items()}
    refs, preds = tok.tokenize(fmt(key2refs)), tok.tokenize(fmt(key2pred))
    scores = {}
    for sc in (Bleu(n=4), Rouge(), Cider(), Meteor(), Spice()):
        s, _ = sc.compute_score(refs, preds)
        scores[sc.method()] = s
    with open(os.path.join(test_dir, "scores.txt"), "w") as f:
        spider = 0.0
        for name, s in scores.items():
            if name == "Bleu":
                for n in range(4):
                    f.write("Bleu-{}: {:6.4f}\n".format(n + 1, s[n]))
            else:
                f.write("{}: {:6.4f}\n".format(name, s))
                if name in ("CIDEr", "SPICE"):
                    spider += s
        f.write("SPIDEr: {:6.4f}\n".format(spider / 2))
    return scores


def main(argv: Optional[Sequence[str]] = None) -> int:
    ap = argparse.ArgumentParser(description="predict_prompt.py on the MI355X pipeline")
    ap.add_argument("--test_dir", type=str, required=True)
    ap.add_argument("--isbeam", action="store_true")
    ap.add_argument("--magic", action="store_true")
    ap.add_argument("--test_data", type=str, required=True)
    ap.add_argument("--tokenizer", type=str, default=None,
                    help="directory with GPT-2 vocab.json + merges.txt (default: <test_dir>/tokenizer)")
    ap.add_argument("--dtype", choices=["f32", "bf16"], default="f32")
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--device", type=str, default="cuda")
    ap.add_argument("--clap", type=str, default=None,
                    help="--magic: CLAP checkpoint ({'model': ASE state dict}, predict_prompt.py:125)")
    ap.add_argument("--bert_vocab", type=str, default=None, help="--magic: BERT vocab.txt")
    args = ap.parse_args(argv)
    if args.magic and not (args.clap and args.bert_vocab):
        raise SystemExit("--magic needs --clap <checkpoint> and --bert_vocab <vocab.txt>")
    params = load_params(args.test_dir)
    tokenizer = GPT2BPE.from_dir(args.tokenizer or os.path.join(args.test_dir, "tokenizer"))
    dtype = torch.float32 if args.dtype == "f32" else torch.bfloat16
    pipe, _ = build_pipeline(args.test_dir, params, tokenizer, args.isbeam, dtype, args.batch,
                             args.device)
    all_data = safeload.load_pickle(args.test_data)
    if args.magic:
        from transformers import BertTokenizer
        ck = torch.load(args.clap, map_location="cpu", weights_only=True)
        clap_sd = ck["model"] if "model" in ck else ck
        with open(args.bert_vocab, encoding="utf-8") as f:
            vocab = {t.rstrip("\n"): i for i, t in enumerate(f)}
        bert_tok = BertTokenizer(vocab=vocab, do_lower_case=True)
        # the reference applies its module-level params {'beta': 0.2, 'alpha': 0.1} AFTER
        # params.json (predict_prompt.py:19-22, 196-197), so magic decoding always runs with
        # alpha 0.1 / beta 0.2 whatever the checkpoint's params.json says; magic_width does come
        # from params.json (line 140: args.magic_width)
        width, alpha, beta = magic_settings(params)
        key2pred, key2pred_prefix, key2refs = make_preds_magic(
            pipe, tokenizer, all_data, clap_sd, bert_tok, width=width, alpha=alpha, beta=beta)
    else:
        key2pred, key2pred_prefix, key2refs = make_preds(pipe, tokenizer, all_data)
    write_outputs(args.test_dir, key2pred, key2pred_prefix, key2refs)
    return 0


if __name__ == "__main__":
    sys.exit(main())
