"""The measurement tools behind bench.py's roofline fields: whole-step HBM traffic
from rocprofv3 counter passes (tools/pmc_step.py) and per-kernel traffic
(tools/pmc_traffic.py), on small synthetic CSVs with known answers.  CPU only."""
import csv
import json
import os
import subprocess
import sys

from conftest import ROOT


def _write_csv(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def _counters(root, name_kib):
    """p1 = FETCH_SIZE, p2 = WRITE_SIZE; name_kib: {kernel: (fetch_kib, write_kib, dispatches)}"""
    for i, cname in enumerate(("FETCH_SIZE", "WRITE_SIZE")):
        rows = []
        for k, (fk, wk, n) in name_kib.items():
            rows += [[k, cname, fk if i == 0 else wk]] * n
        _write_csv(os.path.join(root, f"p{i + 1}", "run_counter_collection.csv"),
                   ["Kernel_Name", "Counter_Name", "Counter_Value"], rows)


def test_pmc_step_sums_one_steady_step(tmp_path):
    pmc = tmp_path / "pmc"
    _counters(str(pmc), {"gemm": (100.0, 50.0, 4), "dw": (10.0, 10.0, 6), "ctn::adam_kernel": (1.0, 1.0, 3)})
    # trace: warm-up kernels, then two steps each [gemm, dw, dw, adam]; the steady step is
    # the dispatches after the second-to-last Adam up to the last one
    seq = ["dw", "ctn::adam_kernel"] + ["gemm", "dw", "dw", "ctn::adam_kernel"] * 2
    rows = [[name, t * 10, t * 10 + 5] for t, name in enumerate(seq)]
    trace = tmp_path / "trace.csv"
    _write_csv(str(trace), ["Kernel_Name", "Start_Timestamp", "End_Timestamp"], rows)
    out = tmp_path / "step.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_step.py"), str(pmc), str(trace), "1.0",
                        str(out)], capture_output=True, text=True, check=True)
    d = json.loads(out.read_text())
    # per launch: gemm (2*100 + 50) KiB, dw (2*10 + 10) KiB, adam (2*1 + 1) KiB
    want = (250 + 2 * 30 + 3) * 1024
    assert abs(d["step_bytes"] - want) < 1e-6
    assert d["kernels"]["dw"]["launches_per_step"] == 2
    assert "step HBM traffic" in r.stdout


def test_pmc_traffic_per_launch(tmp_path):
    pmc = tmp_path / "pmc"
    name = "void ctn::(anonymous namespace)::gemm_dual_ws_kernel<0, 6, 5, false>(ctn::GemmDual)"
    _counters(str(pmc), {name: (1000.0, 400.0, 2)})
    out = tmp_path / "t.json"
    subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(pmc), str(out)], check=True,
                   capture_output=True)
    d = json.loads(out.read_text())
    assert d["3"]["bytes"] == (2 * 1000 + 400) * 1024
    assert d["3"]["launches"] == 2
