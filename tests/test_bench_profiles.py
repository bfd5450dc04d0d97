"""The counter evidence the bench line quotes describes the launch it divides
by: tools/profile_summary.py keeps whole launches only,
and bench.py refuses a summary of another key count or launch shape."""

import csv
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

COLS = ["Correlation_Id", "Dispatch_Id", "Agent_Id", "Queue_Id", "Process_Id", "Thread_Id", "Grid_Size",
        "Kernel_Id", "Kernel_Name", "Workgroup_Size", "LDS_Block_Size", "Scratch_Size", "VGPR_Count",
        "Accum_VGPR_Count", "SGPR_Count", "Counter_Name", "Counter_Value", "Start_Timestamp", "End_Timestamp"]
K = "void lcd::k_spec<2, 2, true, false>(lcd::T0Args)"


def write_pass(path, counter, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, COLS)
        w.writeheader()
        for i, (name, grid, val) in enumerate(rows):
            w.writerow({c: 0 for c in COLS} | {"Dispatch_Id": i + 1, "Grid_Size": grid, "Kernel_Name": name,
                                                "Workgroup_Size": 128, "Counter_Name": counter,
                                                "Counter_Value": val})


def run(args):
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "profile_summary.py")] + args,
                          check=True, capture_output=True, text=True)


def test_whole_launches_only(tmp_path):
    whole, chunk = 128 * 12756, 128 * 3380
    # two whole-shard launches and eight chunk launches of the same kernel,
    # plus another kernel: the median must be over the whole launches
    rows_f = [(K, whole, 75000.0), (K, whole, 76000.0)] + [(K, chunk, 18000.0)] * 8 + [("k_other", whole * 2, 1.0)]
    rows_w = [(K, whole, 8000.0), (K, whole, 8000.0)] + [(K, chunk, 2000.0)] * 8
    f, w = tmp_path / "f.csv", tmp_path / "w.csv"
    write_pass(f, "FETCH_SIZE", rows_f)
    write_pass(w, "WRITE_SIZE", rows_w)
    out = tmp_path / "p.json"
    run(["bytes", "--kernel", "k_spec<2, 2", "--workload", "C3", "--keys", "12500", "--budget", "1048576",
         "--round", "5", "--out", str(out), str(f), str(w)])
    d = json.load(open(out))
    assert d["grid_size"] == whole and d["workgroups"] == 12756
    assert d["dispatches_kept"] == 2 and d["dispatches_total"] == 10
    assert d["bytes_per_launch"] == int(round((2 * 75500.0 + 8000.0) * 1024))
    assert bench.profile_mismatch(d, 12500, d["kernel"]) is None
    assert "keys" in bench.profile_mismatch(d, 1000, d["kernel"])


def test_sq_over_passes(tmp_path):
    whole, chunk = 128 * 12756, 128 * 3380
    p1, p2 = tmp_path / "s1.csv", tmp_path / "s2.csv"
    write_pass(p1, "SQ_INSTS_VALU", [(K, whole, 1.6e9), (K, chunk, 4e8), (K, whole, 1.6e9)])
    write_pass(p2, "SQ_INSTS_SALU", [(K, chunk, 3e8), (K, whole, 1.4e9)])
    out = tmp_path / "s.json"
    run(["sq", "--kernel", "k_spec", "--workload", "C3", "--keys", "12500", "--budget", "1048576", "--round", "5",
         "--out", str(out), str(p1), str(p2)])
    d = json.load(open(out))
    assert d["sq_insts_valu_per_launch"] == 1.6e9 and d["sq_insts_salu_per_launch"] == 1.4e9
    assert d["dispatches_kept"] == 3


def test_refuses_mixed_or_chunk_profiles():
    # round 4's summaries recorded no grid: a median over mixed dispatches
    assert "whole-launch" in bench.profile_mismatch({"keys": 12500}, 12500, K)
    # a chunk-sized launch of the register tier (fewer workgroups than keys)
    d = {"keys": 12500, "whole_launch": True, "grid_size": 128 * 3380, "workgroups": 3380}
    assert "chunk" in bench.profile_mismatch(d, 12500, K)
    # persistent kernels (T3L, WGL) are not held to one workgroup per key
    d = {"keys": 256, "whole_launch": True, "grid_size": 1024 * 256, "workgroups": 256}
    assert bench.profile_mismatch(d, 256, "k_search_layers") is None


def test_probe_rates():
    r = bench.probe_rates(1000, 0, 0.5, 0.0, [], None)
    assert r == {"t0": 1000 / 0.5e-3}
    r = bench.probe_rates(1000, 600, 0.5, 2.0, [2.0], {"probes": 50, "ms_per_launch": 1.0})
    assert r["t0"] == 400 / 0.5e-3 and r["t3"] == 600 / 2e-3 and r["wgl"] == 50 / 1e-3
    assert bench.probe_rates(None, None, 0.0, 0.0, [], None) is None
