#!/usr/bin/env python3
"""Train paper-config Conv-TasNet weights on one MI355X through the HIP training step,
for the separating paper-config parity fixture (tests/golden/make_golden_paper_trained.py).

Paper config (N=256 L=20 B=256 H=512 P=3 X=8 R=4 gLN, 2 speakers; --config c4: the
causal cLN variant with L=16 on 1 s @ 16 kHz mixtures, BASELINE.json configs[3]), bf16 activations,
the solver's update (clip_grad_norm_(5) + Adam lr 1e-3, src/solver.py:178-186), fresh
synthetic speech-like mixtures of 1 s @ 8 kHz every step (synthetic.speech_like, seed =
step).  Writes the fp32 state_dict (torch.save) and a progress log under --out.

    python tools/train_paper_fixture.py --steps 4000 --out gpurun_out/train
    python tools/train_paper_fixture.py --config c4 --steps 3000 --out gpurun_out/train_c4
"""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conv-tasnet_amd"))

import conv_tasnet as ct  # noqa: E402
import ctn_optim  # noqa: E402
import pit_criterion as pc  # noqa: E402
import synthetic  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", choices=("c2", "c4"), default="c2")
    ap.add_argument("--steps", type=int, default=4000)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--samples", type=int, default=None, help="default: 1 s at the config's rate")
    ap.add_argument("--lr", type=float, default=1e-3)
    ap.add_argument("--out", default="gpurun_out/train")
    args = ap.parse_args()
    os.makedirs(args.out, exist_ok=True)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    if args.config == "c4":
        model = ct.ConvTasNet(256, 16, 256, 512, 3, 8, 4, 2, norm_type="cLN", causal=True).to(dev)
        args.samples = args.samples or 16000
    else:
        model = ct.ConvTasNet(256, 20, 256, 512, 3, 8, 4, 2).to(dev)
        args.samples = args.samples or 8000
    model.act_dtype = torch.bfloat16
    opt = ctn_optim.Adam(model.parameters(), lr=args.lr)
    lens = torch.full((args.batch,), args.samples, dtype=torch.int64, device=dev)
    log = open(os.path.join(args.out, "train.log"), "w")
    t0, run = time.time(), 0.0
    nxt = synthetic.speech_like(args.batch, 2, args.samples, 0)
    for step in range(args.steps):
        mix, src = (x.to(dev, non_blocking=True) for x in nxt)
        est = model(mix)
        loss = pc.cal_loss(src, est, lens)[0]
        opt.zero_grad(set_to_none=True)
        loss.backward()
        ctn_optim.clip_grad_norm_(model.parameters(), 5.0)
        opt.step()
        nxt = synthetic.speech_like(args.batch, 2, args.samples, step + 1)   # host work overlaps the GPU
        if step % 100 == 99 or step == args.steps - 1:
            run = float(loss)
            line = f"step {step + 1} loss {run:.4f} ({time.time() - t0:.1f} s)"
            print(line, flush=True)
            log.write(line + "\n")
            log.flush()
    sd = {k: v.detach().float().cpu() for k, v in model.state_dict().items()}
    torch.save(sd, os.path.join(args.out, "paper_weights.pt" if args.config == "c2" else "c4_weights.pt"))
    print(f"saved {len(sd)} tensors, final loss {run:.4f}", flush=True)


if __name__ == "__main__":
    main()
