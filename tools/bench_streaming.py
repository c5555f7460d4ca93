#!/usr/bin/env python3
"""Streaming causal separation (conv-tasnet_amd/streaming.py) latency and throughput
on one MI355X: BASELINE.json's causal configuration (paper dims, causal cLN, L=16,
16 kHz), random weights, fp32 stream kernels.  For each (streams M, chunk of F
frames = F*8 samples): the median wall time of one push() (synchronized, i.e. the
latency from a chunk's arrival to its separated samples on the device) and the
real-time factor (wall time / audio time of the chunk) over 60 pushes after 10 warm-up
pushes.  Prints one JSON object.

    python tools/bench_streaming.py [--out profiles/r03/streaming.json]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "conv-tasnet_amd"))

import conv_tasnet as ct  # noqa: E402
import streaming  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--streams", default="1,16,64", help="comma-separated stream counts")
    ap.add_argument("--frames", default="1,4,16,64", help="comma-separated chunk sizes in frames")
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = ct.ConvTasNet(256, 16, 256, 512, 3, 8, 4, 2, norm_type="cLN", causal=True).to(dev).eval()
    rate, stride = 16000, 8
    rows = []
    for M in [int(v) for v in args.streams.split(",")]:
        for F in [int(v) for v in args.frames.split(",")]:
            s = streaming.StreamingSeparator(model)
            n = F * stride
            x = torch.randn(M, n * 70 + 16, device=dev)
            s.push(x[:, :16])                     # the first frame's overlap
            times = []
            for i in range(70):
                chunk = x[:, 16 + i * n:16 + (i + 1) * n]
                torch.cuda.synchronize(dev)
                t0 = time.perf_counter()
                s.push(chunk)
                torch.cuda.synchronize(dev)
                if i >= 10:
                    times.append(time.perf_counter() - t0)
            times.sort()
            med = times[len(times) // 2]
            audio = n / rate
            rows.append({"streams": M, "chunk_frames": F, "chunk_ms_audio": round(audio * 1e3, 3),
                         "latency_ms_median": round(med * 1e3, 3), "latency_ms_p90": round(times[int(len(times) * 0.9)] * 1e3, 3),
                         "real_time_factor": round(med / audio, 4),
                         "stream_seconds_per_second": round(M * audio / med, 2)})
            print(json.dumps(rows[-1]), flush=True)
    out = {"model": "paper dims causal cLN, L=16 @ 16 kHz (BASELINE.json configs[3]), random weights, fp32 stream "
                    "kernels (csrc/ctn_stream.hip)", "rows": rows}
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
