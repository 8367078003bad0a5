"""The profile summarisers the BASELINE numbers come from, on synthetic rocprofv3 CSVs:
scripts/summarize_trace.py (timed window between the marker kernels, busy / idle accounting,
per-class shares, kernels outside the HIP library) and scripts/gemm_pmc_table.py (effective
clock = GRBM_GUI_ACTIVE / 8 / duration, MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (1024 x cycles))."""
import csv
import importlib.util
import io
import os
from contextlib import redirect_stdout

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load(name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, "scripts", f"{name}.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write(path, header, rows):
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=header)
        w.writeheader()
        for r in rows:
            w.writerow(r)


def test_summarize_trace_window_and_foreign_kernels(tmp_path):
    st = _load("summarize_trace")
    us = 1000  # ns
    rows = [
        ("warmup_kernel", 0, 50),                       # before the window: excluded
        ("lk_window_mark_kernel", 100, 101),
        ("void anon::gemm_kernel<4, 1>(x)", 110, 610),  # 500 us
        ("void anon::paged_decode_kernel<128, 4>(x)", 620, 720),
        ("void at::native::vectorized_elementwise_kernel<4>(x)", 900, 910),  # 180 us gap before
        ("__amd_rocclr_copyBuffer", 910, 920),
        ("lk_window_mark_kernel", 1100, 1101),
        ("drain_kernel", 1200, 1300),                   # after the window: excluded
    ]
    path = tmp_path / "run_kernel_trace.csv"
    _write(path, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"],
           [{"Kernel_Name": n, "Start_Timestamp": s * us, "End_Timestamp": e * us} for n, s, e in rows])
    buf = io.StringIO()
    with redirect_stdout(buf):
        st.main(str(path), 4.0)
    out = buf.getvalue()
    assert "between the lk_window_mark kernels" in out
    assert "warmup_kernel" not in out and "drain_kernel" not in out
    assert "4 kernels" in out
    assert "| prefill GEMM (gemm_kernel / gemm1w, MFMA) | 0.5 |" in out
    # the 180 us gap is itemised with the kernels on either side
    assert "| 180 |" in out
    # kernels outside the HIP library: the eager PyTorch op and the runtime copy, not ours
    foreign = out.split("kernel outside the HIP library")[1].split("\n\n")[0]
    assert "at::native" in foreign and "copyBuffer" in foreign
    assert "gemm_kernel" not in foreign and "paged_decode" not in foreign


def test_gemm_pmc_table_clock_and_mfma_busy(tmp_path):
    gp = _load("gemm_pmc_table")
    d = tmp_path / "o_4096_4096_4096_prod" / "host"
    d.mkdir(parents=True)
    kt, cc = [], []
    dur_us, ghz, busy = 100.0, 2.0, 0.6
    cycles = dur_us * 1e3 * ghz  # shader cycles in the dispatch
    for i in range(8):
        s = i * 1_000_000
        kt.append({"Dispatch_Id": i, "Kernel_Name": "gemm_kernel", "Start_Timestamp": s,
                   "End_Timestamp": s + int(dur_us * 1e3)})
        for name, val in (("GRBM_GUI_ACTIVE", 8 * cycles), ("SQ_VALU_MFMA_BUSY_CYCLES", busy * 1024 * cycles),
                          ("SQ_WAIT_ANY", 30.0), ("SQ_WAVE_CYCLES", 100.0), ("SQ_INSTS_MFMA", 1.0)):
            cc.append({"Dispatch_Id": i, "Kernel_Name": "gemm_kernel", "Counter_Name": name, "Counter_Value": val})
    _write(d / "run_kernel_trace.csv", ["Dispatch_Id", "Kernel_Name", "Start_Timestamp", "End_Timestamp"], kt)
    _write(d / "run_counter_collection.csv", ["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"], cc)
    r = gp.load(str(tmp_path / "o_4096_4096_4096_prod"))
    assert r["dispatches"] == 3  # the first 5 are warm-up
    assert abs(r["us"] - dur_us) < 1e-6
    assert abs(r["clock_ghz"] - ghz) < 1e-9
    assert abs(r["mfma_busy"] - busy) < 1e-9
    assert abs(r["wait_share"] - 0.3) < 1e-9
    md = tmp_path / "t.md"
    buf = io.StringIO()
    with redirect_stdout(buf):
        import sys
        argv, sys.argv = sys.argv, ["gemm_pmc_table.py", str(tmp_path / "o_4096_4096_4096_prod"), "--md", str(md)]
        try:
            gp.main()
        finally:
            sys.argv = argv
    row = md.read_text().splitlines()[2]
    # 2 * 4096^3 FLOP in 100 us = 1374 TF/s; busy x clock = 1.2
    assert "| 1374 |" in row and "| 2.00 |" in row and "60.0 %" in row and "| 1.200 |" in row


def test_attn_phase_splits_overlap(tmp_path):
    """scripts/attn_phase.py: a mixed step's attention phase (first attention kernel after a GEMM
    to the next GEMM) split into both-running / flash-only / decode-only / neither."""
    ap = _load("attn_phase")
    us = 1000
    rows = [
        ("lk_window_mark_kernel", 0, 1),
        ("void anon::gemm1w_kernel<7, 16, 256, false>(x)", 10, 100),   # QKV
        ("void anon::flash_prefill_kernel<128, true>(x)", 100, 160),    # flash 100-160
        ("void anon::paged_decode_kernel<128, 4>(x)", 120, 200),       # decode 120-200
        ("void anon::gemm1w_kernel<6, 0, 256, false>(x)", 210, 300),    # O: phase ends at 210
        ("void anon::paged_decode_kernel<128, 4>(x)", 300, 350),       # a decode-only phase
        ("void anon::wsgemm_kernel<12, 128, false>(x)", 355, 400),
        ("lk_window_mark_kernel", 500, 501),
    ]
    path = tmp_path / "run_kernel_trace.csv"
    _write(path, ["Kernel_Name", "Start_Timestamp", "End_Timestamp"],
           [{"Kernel_Name": n, "Start_Timestamp": s * us, "End_Timestamp": e * us} for n, s, e in rows])
    ph = ap.phases(list(csv.DictReader(open(path))))
    assert len(ph) == 2
    mixed = ph[0]
    assert mixed["next_gemm"] - mixed["start"] == 110 * us
    f, d = ap._union(mixed["flash"]), ap._union(mixed["decode"])
    both = ap._len(ap._inter(f, d))
    assert both == 40 * us                       # 120-160
    assert ap._len(f) - both == 20 * us          # flash alone 100-120
    assert ap._len(d) - both == 40 * us          # decode alone 160-200
    assert ph[1]["decode"] and not ph[1]["flash"]
    buf = io.StringIO()
    with redirect_stdout(buf):
        import sys
        argv = sys.argv
        sys.argv = ["attn_phase.py", str(path)]
        try:
            ap.main()
        finally:
            sys.argv = argv
    out = buf.getvalue()
    assert "mixed (flash + decode): 1 phases" in out and "decode only: 1 phases" in out
