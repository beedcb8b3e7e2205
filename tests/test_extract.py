"""Host side of the batched embedding extractor (zsaac/extract.py, the reference's
Extract_embeddings, data_handing/embeddings_generator.py:34-75, 100-101): which clips are
encoded and with how many samples, the record format, and the pickle location / round trip
through the allow-list loader the predict harness uses."""
import os

import torch


def test_fit_plan_crop_pad_skip():
    from zsaac.extract import fit_plan
    keep, kept = fit_plan([800000, 0, 128000, 320000, 1], 320000)
    assert keep == [0, 2, 3, 4]                 # the empty clip is skipped (line 50-51)
    assert kept == [320000, 128000, 320000, 1]   # crop to the first T, else keep all (pad rest)


def test_records_and_pickle_roundtrip(tmp_path):
    from zsaac import safeload
    from zsaac.extract import make_record, save_records
    emb = torch.randn(3, 1024)
    recs = [make_record(emb[i], [f"cap {i}", "other"], f"clip{i}") for i in range(3)]
    assert recs[0]["audio_embedding"].shape == (1, 1024) and recs[0]["text_embedding"] == 0
    path = save_records(recs, str(tmp_path), "test")
    assert path == os.path.join(str(tmp_path), "test", "clap_embedding", "ZS", "data.pkl")
    back = safeload.load_pickle(path)
    assert [r["audio_id"] for r in back] == ["clip0", "clip1", "clip2"]
    assert torch.equal(back[1]["audio_embedding"], emb[1:2])
    assert back[2]["caption"] == ["cap 2", "other"]
