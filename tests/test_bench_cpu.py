"""bench.py's host-side helpers (no GPU): kernel-function grouping of census names, the rocprof
name mapping the PMC traffic files are keyed by, and the PMC traffic reduction of
tools/pmc_traffic.py on a synthetic counter file (FETCH_SIZE x 2 on gfx950 + WRITE_SIZE, KiB)."""
import csv
import importlib.util
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_kernel_names():
    b = _bench()
    assert b.kernel_function("conv3x3_gn_p4_kernel<32>") == "conv3x3_gn_p4_kernel"
    assert b.kernel_function("(conv_pipe<T, 2, true>)") == "conv_pipe"
    assert b.rocprof_name("(conv_pipe<T, 2, true>)") == "conv_pipe<unsigned short, 2, true>"
    assert b.kernel_file("conv3x3_gn_p4_kernel<16>") == "conv3x3_gn_p4_kernel_16"


def test_pmc_traffic_reduction(tmp_path):
    d = tmp_path / "pmc"
    rows = []
    # two dispatches of the <32> instantiation (template defaults printed by rocprof), one of <16>
    for did, name, fetch, write in [(1, "void itsd::conv3x3_gn_p4_kernel<32, 0, false>(itsd::ConvArgs)", 100.0, 40.0),
                                    (2, "void itsd::conv3x3_gn_p4_kernel<16, 0, false>(itsd::ConvArgs)", 7.0, 3.0),
                                    (3, "void itsd::conv3x3_gn_p4_kernel<32, 0, false>(itsd::ConvArgs)", 120.0, 60.0)]:
        rows.append((f"p0", did, name, "FETCH_SIZE", fetch))
        rows.append((f"p1", did, name, "WRITE_SIZE", write))
    for sub in ("p0", "p1"):
        (d / sub).mkdir(parents=True)
        with open(d / sub / "run_counter_collection.csv", "w", newline="") as fh:
            w = csv.DictWriter(fh, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
            w.writeheader()
            for s, did, name, ctr, v in rows:
                if s == sub:
                    w.writerow({"Dispatch_Id": did, "Kernel_Name": name, "Counter_Name": ctr, "Counter_Value": v})
    out = tmp_path / "t.json"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_traffic.py"), str(d),
                        "conv3x3_gn_p4_kernel<32>", str(out)], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    t = json.load(open(out))
    assert t["launches"] == 2
    # per launch: mean over the two dispatches of (FETCH x 2 + WRITE), KiB -> bytes
    want = ((100 * 2 + 40) + (120 * 2 + 60)) / 2 * 1024
    assert abs(t["hbm_bytes_per_launch"] - want) < 1e-6


def test_cpu_baseline_conversion_check_fields():
    """The CPU baseline's conversion check is a check: equal interleaved windows of the full N = 1
    loop and of B = 1 forwards, a deviation, and `agrees` within +-15 % (tiny windows here)."""
    b = _bench()
    r = b.cpu_baseline(1000, seconds=0.6, check_seconds=0.8)
    c = r["full_loop_check"]
    assert r["kind"] == "port" and r["cores"] >= 1 and r["value"] > 0
    assert len(c["loop_steps_per_s"]) == 2 and len(c["b1_fwd_per_s"]) == 2
    dev = (max(c["loop_steps_per_s"]) - max(c["b1_fwd_per_s"])) / max(c["b1_fwd_per_s"])
    # (the rates in the record are rounded to 3 decimals: at a few steps/s on a loaded host that alone moves
    # the recomputed deviation by ~1e-3)
    assert abs(c["deviation"] - dev) < 5e-3 and c["agrees"] == (abs(c["deviation"]) <= 0.15)


def test_conv_alg_bytes_counts_every_operand_once():
    """the algorithmic bytes of a fused conv launch count the residual operand and the
    GroupNorm statistics slabs (output written, fused input read), besides input, weights and output."""
    import bench
    M, N, K = 256 * 1024, 128, 9 * 128
    o = {"M": M, "N": N, "K": K, "H": 32, "ks": 3, "stride_up": 10, "resid": False, "stats_out": False, "gn_in": False}
    base = 2.0 * (M * 128 + N * K + M * N)
    assert bench.conv_alg_bytes(o) == base
    o.update(resid=True, stats_out=True, gn_in=True)
    slots = M / 128  # 128-pixel statistics slots of the 32x32 images
    assert bench.conv_alg_bytes(o) == base + 2.0 * M * N + 8.0 * slots * N + 8.0 * slots * 128
    # nearest-x2 upsample conv (input grid a quarter of the output's), 4x4 level slots of 16 pixels
    up = {"M": 4096, "N": 512, "K": 9 * 512, "H": 8, "ks": 3, "stride_up": 11, "resid": False, "stats_out": True,
          "gn_in": False}
    assert bench.conv_alg_bytes(up) == 2.0 * (1024 * 512 + 512 * 9 * 512 + 4096 * 512) + 8.0 * (4096 / 64) * 512
