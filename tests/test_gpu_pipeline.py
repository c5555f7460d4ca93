"""End to end on the HIP path: wav corpus ->
preprocess manifests -> train (Solver: checkpoints, best model) -> resume ->
evaluate (SI-SNRi) -> separate (PCM_16 wavs), on a small model.  GPU only."""
import json
import os
import types

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

SR = 8000


def _corpus(root, seed=0):
    """tr/cv/tt splits of 2-speaker mixtures (speech-like sources, varied lengths)."""
    import synthetic
    from audio_io import write_wav
    lengths = {"tr": [6400, 9000, 4000, 12000, 7000, 5000], "cv": [6000, 9500], "tt": [5000, 7300]}
    for split, lens in lengths.items():
        for d in ("mix", "s1", "s2"):
            os.makedirs(os.path.join(root, "wav", split, d), exist_ok=True)
        for i, n in enumerate(lens):
            mix, src = synthetic.speech_like(1, 2, n, seed + 31 * i + len(split))
            scale = 0.3 / float(mix.abs().max())
            write_wav(os.path.join(root, "wav", split, "mix", f"u{i}.wav"), mix[0].numpy() * scale, SR)
            for c in range(2):
                write_wav(os.path.join(root, "wav", split, f"s{c + 1}", f"u{i}.wav"), src[0, c].numpy() * scale, SR)


def _train_args(root, **kw):
    import train
    a = train.parser.parse_args([
        "--train_dir", os.path.join(root, "json", "tr"), "--valid_dir", os.path.join(root, "json", "cv"),
        "--N", "64", "--L", "20", "--B", "64", "--H", "128", "--P", "3", "--X", "2", "--R", "2",
        "--segment", "0.5", "--batch_size", "6", "--num_workers", "0", "--epochs", "2", "--checkpoint", "1",
        "--save_folder", os.path.join(root, "exp"), "--print_freq", "1", "--lr", "1e-3"])
    for k, v in kw.items():
        setattr(a, k, v)
    return a


def test_preprocess_train_resume_evaluate_separate(tmp_path):
    import evaluate
    import preprocess
    import separate
    import train
    root = str(tmp_path)
    _corpus(root)
    preprocess.preprocess(types.SimpleNamespace(in_dir=os.path.join(root, "wav"), out_dir=os.path.join(root, "json"),
                                                sample_rate=SR))
    assert len(json.load(open(os.path.join(root, "json", "tr", "mix.json")))) == 6

    torch.manual_seed(0)
    train.main(_train_args(root))
    exp = os.path.join(root, "exp")
    assert {"epoch1.pth.tar", "epoch2.pth.tar", "final.pth.tar"} <= set(os.listdir(exp))
    pkg = torch.load(os.path.join(exp, "epoch2.pth.tar"), weights_only=True)
    assert pkg["epoch"] == 2 and np.isfinite(float(pkg["tr_loss"][0]))
    assert set(pkg["optim_dict"]["state"]) and pkg["optim_dict"]["param_groups"][0]["lr"] == 1e-3

    # resume for one more epoch (solver.py:50-59)
    train.main(_train_args(root, epochs=3, continue_from=os.path.join(exp, "epoch2.pth.tar")))
    assert "epoch3.pth.tar" in os.listdir(exp)
    pkg3 = torch.load(os.path.join(exp, "epoch3.pth.tar"), weights_only=True)
    assert pkg3["epoch"] == 3 and float(pkg3["tr_loss"][1]) == float(pkg["tr_loss"][1])

    model_path = os.path.join(exp, "final.pth.tar")
    v = evaluate.evaluate(evaluate.parser.parse_args(["--model_path", model_path, "--data_dir",
                                                      os.path.join(root, "json", "tt"), "--batch_size", "2",
                                                      "--num_workers", "0"]))
    assert np.isfinite(v)

    out = os.path.join(root, "sep")
    separate.separate(separate.parser.parse_args(["--model_path", model_path, "--mix_dir",
                                                  os.path.join(root, "wav", "tt", "mix"), "--out_dir", out]))
    from audio_io import read_wav
    for i, n in enumerate((5000, 7300)):
        for suffix in ("", "_s1", "_s2"):
            y, sr = read_wav(os.path.join(out, f"u{i}{suffix}.wav"))
            assert sr == SR and len(y) == n


def test_evaluate_matches_numpy_reference_metric(tmp_path):
    """The batched device SI-SNRi equals the reference's per-utterance numpy metric
    (evaluate.py:108-144) on a model's reordered estimates, ragged lengths included."""
    import conv_tasnet as ct
    import evaluate
    import pit_criterion as pc
    from utils import remove_pad
    torch.manual_seed(0)
    model = ct.ConvTasNet(64, 20, 64, 128, 3, 2, 2, 2).cuda().eval()
    import synthetic
    mix, src = synthetic.speech_like(3, 2, 8000, 7)
    lens = torch.tensor([8000, 6100, 3333])
    for b in range(3):
        mix[b, lens[b]:] = 0
        src[b, :, lens[b]:] = 0
    mix, src, lens = mix.cuda(), src.cuda(), lens.cuda()
    with torch.no_grad():
        est = model(mix)
        _, _, est, reord = pc.cal_loss(src, est, lens)
    got = evaluate.cal_SISNRi_batch(src, reord, mix, lens).cpu().numpy()
    for b, (m, s, e) in enumerate(zip(remove_pad(mix, lens), remove_pad(src, lens), remove_pad(reord, lens))):
        assert got[b] == pytest.approx(evaluate.cal_SISNRi(s.astype(np.float64), e.astype(np.float64),
                                                           m.astype(np.float64)), abs=1e-6)
