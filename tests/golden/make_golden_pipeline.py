"""Golden vectors for the data pipeline and the solver's epoch control
(SURVEY.md §8f rows 1-3), captured from the REAL reference (build container only).

Run from the repo root:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_pipeline.py

It imports jwr1995/Conv-TasNet from /root/reference/src (read-only).  librosa
is not installed, so ``librosa.load`` is replaced by a deterministic synthetic
signal per path (``synth_signal``, length from the manifest): the captured
vectors pin the reference's bucketing, segmentation, padding and collate logic
(data.py); wav decoding is pinned separately by known-answer tests
(tests/test_pipeline.py).  The Solver (solver.py) runs with its per-epoch pass
replaced by a scripted loss sequence, which pins the LR-halving / early-stop /
checkpoint rules of solver.py:69-156 (also when resuming from a checkpoint).
Only manifests, numbers and file names are written: pipeline.json, pipeline.npz.
"""
import json
import os
import sys
import tempfile
import types
import zlib

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, "/root/reference/src")
torch.Tensor.cuda = lambda self, *a, **k: self          # utils.py:40 shim

LENGTHS = {}


def synth_signal(path, n):
    rng = np.random.default_rng(zlib.crc32(path.encode()))
    return (0.1 * rng.standard_normal(n)).astype(np.float32)


def _fake_load(path, sr=None, **kw):
    return synth_signal(path, LENGTHS[path]), sr


_librosa = types.ModuleType("librosa")
_librosa.load = _fake_load
sys.modules["librosa"] = _librosa

import conv_tasnet as ref_ct      # noqa: E402
import data as ref_data          # noqa: E402
import solver as ref_solver      # noqa: E402

SR = 50                          # 4 s segments = 200 samples: small fixtures


def manifest(n_utt, seed, lo, hi, split):
    rng = np.random.default_rng(seed)
    lens = [int(v) for v in rng.integers(lo, hi, n_utt)]
    lens[3] = lens[5]            # ties: the stable sort keeps manifest order
    lens[7] = lens[8] = 4 * SR   # exactly one segment
    lens[10] = 2 * 4 * SR        # exactly two segments
    infos = {name: [[f"{split}/{name}/u{i:03d}.wav", n] for i, n in enumerate(lens)] for name in ("mix", "s1", "s2")}
    for lst in infos.values():
        for p, n in lst:
            LENGTHS[p] = n
    return infos


def write_manifest(d, infos):
    for name, lst in infos.items():
        with open(os.path.join(d, name + ".json"), "w") as f:
            json.dump(lst, f)


def data_fixtures(out, arrays):
    tr = manifest(40, 1, 60, 1700, "tr")
    out["tr_infos"] = tr
    cases = []
    with tempfile.TemporaryDirectory() as d:
        write_manifest(d, tr)
        for bs, seg, cvmax in [(1, 4.0, 8.0), (3, 4.0, 8.0), (7, 4.0, 8.0), (20, 4.0, 8.0),
                               (3, -1, 8.0), (4, -1, 30.0), (1, -1, 20.0)]:
            ds = ref_data.AudioDataset(d, bs, sample_rate=SR, segment=seg, cv_maxlen=cvmax)
            key = f"bs{bs}_seg{seg}_cv{cvmax}"
            cases.append({"key": key, "batch_size": bs, "segment": seg, "cv_maxlen": cvmax,
                          "minibatch": ds.minibatch})
            if key in ("bs7_seg4.0_cv8.0", "bs3_seg-1_cv8.0"):
                for i in range(min(5, len(ds))):
                    mix, ilens, src = ref_data._collate_fn([ds[i]])
                    arrays[f"{key}.{i}.mix"] = mix.numpy()
                    arrays[f"{key}.{i}.ilens"] = ilens.numpy()
                    arrays[f"{key}.{i}.src"] = src.numpy()
        # evaluation dataset (mixtures only, from a manifest)
        ev = ref_data.EvalDataset(None, os.path.join(d, "mix.json"), 3, sample_rate=SR)
        out["eval_minibatch"] = ev.minibatch
        for i in range(2):
            mix, ilens, names = ref_data._collate_fn_eval([ev[i]])
            arrays[f"eval.{i}.mix"] = mix.numpy()
            arrays[f"eval.{i}.ilens"] = ilens.numpy()
            out[f"eval.{i}.names"] = names
    out["data_cases"] = cases
    xs = [torch.arange(n * 2, dtype=torch.float32).view(n, 2) for n in (3, 5, 1)]
    arrays["pad_list"] = ref_data.pad_list(xs, -1.5).numpy()


class Holder(torch.nn.Module):   # nn.DataParallel stand-in: the solver uses .module
    def __init__(self, m):
        super().__init__()
        self.module = m


def solver_run(folder, tr, cv, epochs, half_lr, early_stop, checkpoint, continue_from=""):
    torch.manual_seed(0)
    model = Holder(ref_ct.ConvTasNet(8, 4, 6, 10, 3, 2, 1, 2))
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    args = types.SimpleNamespace(use_cuda=0, epochs=epochs, half_lr=half_lr, early_stop=early_stop, max_norm=5.0,
                                 save_folder=folder, checkpoint=checkpoint, continue_from=continue_from,
                                 model_path="final.pth.tar", print_freq=10, visdom=0, visdom_epoch=0,
                                 visdom_id="golden")
    s = ref_solver.Solver({"tr_loader": None, "cv_loader": None}, model, opt, args)
    trace, it_tr, it_cv = [], iter(tr), iter(cv)

    def scripted(epoch, cross_valid=False):
        if cross_valid:
            return next(it_cv)
        trace.append([epoch, opt.param_groups[0]["lr"]])
        return next(it_tr)

    s._run_one_epoch = scripted
    s.train()
    files = sorted(os.listdir(folder))
    pk = {}
    for f in files:
        p = torch.load(os.path.join(folder, f), weights_only=True)
        n = int(p["epoch"])
        valid = n if f == "final.pth.tar" else n - 1   # epoch files are written before their losses
        pk[f] = {"epoch": n, "tr_loss": p["tr_loss"][:valid].tolist(), "cv_loss": p["cv_loss"][:valid].tolist(),
                 "lr": p["optim_dict"]["param_groups"][0]["lr"]}
    return {"trace": trace, "files": files, "packages": pk, "final_lr": opt.param_groups[0]["lr"]}


SOLVER_CASES = {
    # halving after 3 non-improving epochs, early stop after 10, checkpoints on
    "halve_stop": dict(epochs=30, half_lr=1, early_stop=1, checkpoint=1,
                       cv=[-5.0, -6.0, -7.0, -6.5, -6.4, -6.3, -6.8, -6.7, -6.6, -6.5, -6.4, -6.3, -6.2, -6.1,
                           -6.0, -5.9, -5.8, -5.7, -5.6, -5.5, -5.4, -5.3]),
    # no halving: only the best model is written
    "plain": dict(epochs=5, half_lr=0, early_stop=0, checkpoint=0, cv=[-3.0, -4.0, -3.5, -4.5, -4.4]),
    # halving without early stop, equal losses count as no improvement
    "halve_only": dict(epochs=12, half_lr=1, early_stop=0, checkpoint=0,
                       cv=[-1.0, -1.0, -1.0, -1.0, -2.0, -2.0, -2.0, -2.5, -2.4, -2.3, -2.2, -2.6]),
}


def solver_fixtures(out):
    res = {}
    for name, c in SOLVER_CASES.items():
        tr = [-0.5 * i - 1.0 for i in range(len(c["cv"]))]
        with tempfile.TemporaryDirectory() as d:
            res[name] = solver_run(d, tr, c["cv"], c["epochs"], c["half_lr"], c["early_stop"], c["checkpoint"])
            res[name]["tr"] = tr
            res[name]["cv"] = c["cv"]
            if name == "halve_stop":
                # resume from the epoch-4 checkpoint with a new loss script
                with tempfile.TemporaryDirectory() as d2:
                    cv2 = [-6.6, -6.55, -6.5, -6.45, -6.9, -7.2]
                    tr2 = [-3.0 - 0.1 * i for i in range(len(cv2))]
                    r = solver_run(d2, tr2, cv2, 10, 1, 1, 1, continue_from=os.path.join(d, "epoch4.pth.tar"))
                    r.update(tr=tr2, cv=cv2)
                    res["resume4"] = r
    out["solver"] = res


if __name__ == "__main__":
    out, arrays = {"sample_rate": SR, "torch": torch.__version__}, {}
    data_fixtures(out, arrays)
    solver_fixtures(out)
    with open(os.path.join(HERE, "pipeline.json"), "w") as f:
        json.dump(out, f, indent=1)
    np.savez_compressed(os.path.join(HERE, "pipeline.npz"), **arrays)
    print("wrote pipeline.json / pipeline.npz")
