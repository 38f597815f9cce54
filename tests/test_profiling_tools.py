"""The rocprofv3 post-processing tools the round-5 evidence rests on (bench/step_pmc.py,
bench/wave_efficiency.py, bench/rocprof_rows.py), on small synthetic traces: the last-step cut,
the pass-to-trace join by position (and its refusal on a mismatch), the derived MFMA busy and
byte columns, the resident-block model and the SQLite/CSV row loader."""
import csv
import os
import sqlite3
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))

import rocprof_rows  # noqa: E402
import step_pmc  # noqa: E402
import wave_efficiency  # noqa: E402

# one "step" = conv, bn, sgd; three steps plus a warm-up kernel
KERNELS = ["void dpt::warm_kernel()"] + ["void dpt::conv_fwd_kernel<128>(dpt::ConvFwdArgs)",
                                          "void dpt::bn_fwd_apply_kernel<BF16>()",
                                          "void dpt::sgd_kernel<2>(float*)"] * 3


def _write_trace(d, durations_us):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_kernel_trace.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        w.writeheader()
        t = 1000
        for name, us in zip(KERNELS, durations_us):
            w.writerow({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + int(us * 1000)})
            t += int(us * 1000) + 500


def _write_pass(d, counters, names=KERNELS):
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "run_counter_collection.csv"), "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=["Dispatch_Id", "Kernel_Name", "Counter_Name", "Counter_Value"])
        w.writeheader()
        for i, name in enumerate(names, start=1):
            for k, v in counters(i, name).items():
                w.writerow({"Dispatch_Id": i, "Kernel_Name": name, "Counter_Name": k, "Counter_Value": v})


def test_step_pmc_joins_the_last_step(tmp_path, capsys):
    durs = [5.0] + [100.0, 50.0, 10.0] * 3
    _write_trace(str(tmp_path / "kt"), durs)
    # MFMA busy cycles = half of the CU-SIMD cycles for the conv, none elsewhere
    gui = 8 * 1000.0

    def pa(i, name):
        busy = 0.5 * (gui / 8 * 256 * 4) if "conv" in name else 0.0
        return {"SQ_VALU_MFMA_BUSY_CYCLES": busy, "GRBM_GUI_ACTIVE": gui}

    _write_pass(str(tmp_path / "pA"), pa)
    _write_pass(str(tmp_path / "pB"), lambda i, n: {"FETCH_SIZE": 1.0e6})    # KiB: x2 on the read side
    _write_pass(str(tmp_path / "pC"), lambda i, n: {"WRITE_SIZE": 5.0e5})
    step_pmc.main(["--passes", str(tmp_path / "pA"), str(tmp_path / "pB"), str(tmp_path / "pC"),
                   "--trace", str(tmp_path / "kt")])
    out = capsys.readouterr().out
    assert "3 dispatches" in out                        # the last full step only
    conv = next(l for l in out.splitlines() if "conv_fwd_kernel" in l)
    cells = [c.strip() for c in conv.split("|")]
    # | kernel | calls | us | share | busy | read | write | TB/s | % |
    assert cells[2] == "1" and cells[3] == "100.0" and cells[5] == "50%"
    assert float(cells[6]) == pytest.approx(2 * 1.0e6 * 1024 / 1e9, rel=1e-3)
    assert float(cells[7]) == pytest.approx(5.0e5 * 1024 / 1e9, rel=1e-3)


def test_step_pmc_refuses_a_misaligned_pass(tmp_path):
    _write_trace(str(tmp_path / "kt"), [5.0] + [100.0, 50.0, 10.0] * 3)
    names = list(KERNELS)
    names[-2] = "void dpt::something_else()"            # same count, different kernel at one position
    _write_pass(str(tmp_path / "pA"), lambda i, n: {"GRBM_GUI_ACTIVE": 1.0}, names)
    with pytest.raises(SystemExit, match="dispatch 1"):
        step_pmc.main(["--passes", str(tmp_path / "pA"), "--trace", str(tmp_path / "kt")])


def test_blocks_per_cu_model():
    # 4-wave blocks: LDS-limited (36 KiB -> 4), VGPR-limited (256 regs -> 2), wave cap (8 per SIMD)
    assert wave_efficiency.blocks_per_cu(36864, 64, 0, 256) == 4
    assert wave_efficiency.blocks_per_cu(0, 256, 0, 256) == 2
    assert wave_efficiency.blocks_per_cu(0, 32, 0, 256) == 8
    # 8-wave blocks take two waves per SIMD
    assert wave_efficiency.blocks_per_cu(0, 128, 0, 512) == 2
    # unified register file: arch + accumulation VGPRs add up (granule 8)
    assert wave_efficiency.blocks_per_cu(0, 100, 30, 256) == 512 // 136


def test_rocprof_rows_reads_sqlite_and_csv(tmp_path):
    db = str(tmp_path / "run_results.db")
    c = sqlite3.connect(db)
    cols = list(rocprof_rows._MAP)
    c.execute(f"create table kernels ({', '.join(cols)})")
    vals = {k: 0 for k in cols}
    for name, start in (("b", 20), ("a", 10)):
        v = dict(vals)
        v[cols[0]] = name
        for k, m in rocprof_rows._MAP.items():
            if m == "Start_Timestamp":
                v[k] = start
            elif m == "End_Timestamp":
                v[k] = start + 5
        c.execute(f"insert into kernels values ({', '.join('?' * len(cols))})", [v[k] for k in cols])
    c.commit()
    c.close()
    rows = rocprof_rows.load_rows(db)
    assert [int(r["Start_Timestamp"]) for r in rows] == [10, 20]
    assert set(rocprof_rows._MAP.values()) <= set(rows[0])
    _write_trace(str(tmp_path / "kt"), [1.0] * len(KERNELS))
    rows = rocprof_rows.load_rows(str(tmp_path / "kt" / "run_kernel_trace.csv"))
    assert [r["Kernel_Name"] for r in rows] == KERNELS


def _write_full_trace(path, rows):
    cols = ["Kernel_Name", "Start_Timestamp", "End_Timestamp", "LDS_Block_Size", "VGPR_Count", "Accum_VGPR_Count",
            "Workgroup_Size_X", "Workgroup_Size_Y", "Workgroup_Size_Z", "Grid_Size_X", "Grid_Size_Y", "Grid_Size_Z"]
    with open(path, "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=cols)
        w.writeheader()
        t = 1000
        for name, us, blocks, vgpr_trace, lds in rows:
            w.writerow({"Kernel_Name": name, "Start_Timestamp": t, "End_Timestamp": t + int(us * 1000),
                        "LDS_Block_Size": lds, "VGPR_Count": vgpr_trace, "Accum_VGPR_Count": 0,
                        "Workgroup_Size_X": 256, "Workgroup_Size_Y": 1, "Workgroup_Size_Z": 1,
                        "Grid_Size_X": 256 * blocks, "Grid_Size_Y": 1, "Grid_Size_Z": 1})
            t += int(us * 1000) + 500


def test_wave_efficiency_splits_tail_from_sub_wave_grids(tmp_path, capsys):
    """Round 6: the idle estimate is split into the last-wave tail of grids of >= 1 wave and the
    upper bound from grids smaller than one wave, and the trace's VGPR_Count (half the compiler's
    count on gfx950) is scaled back before the resident-block model."""
    # 64 in the trace = 128 VGPRs -> 4 blocks per CU -> 1024 slots
    rows = [("void dpt::conv_fwd_kernel<1>(x)", 100.0, 1536, 64, 0),    # 1.5 waves: eff 0.75
            ("void dpt::conv_wgrad_kernel<1>(x)", 100.0, 512, 64, 0),   # 0.5 wave: eff 0.5
            ("void dpt::sgd_kernel<2>(float*)", 10.0, 256, 16, 0)] * 2
    p = str(tmp_path / "kt.csv")
    _write_full_trace(p, rows)
    wave_efficiency.main([p, "--steps", "1"])
    out = capsys.readouterr().out
    multi = next(l for l in out.splitlines() if l.startswith("| >= 1 wave"))
    sub = next(l for l in out.splitlines() if l.startswith("| < 1 wave"))
    # last step only: conv 100 us x (1 - 0.75) = 25 us tail; wgrad 100 x 0.5 = 50 us and sgd (256
    # blocks at 8 per CU: 1/8 of a wave) 10 x 0.875 us of upper bound
    assert [c.strip() for c in multi.split("|")][3] == "0.025"
    assert [c.strip() for c in sub.split("|")][3] == "0.059"
    conv = next(l for l in out.splitlines() if "conv_fwd_kernel" in l)
    assert [c.strip() for c in conv.split("|")][3] == "4" and [c.strip() for c in conv.split("|")][5] == "128"


def test_selfcheck_acceptance_rule():
    from distributed_pytorch_training_amd.engine import selfcheck
    ok = {"loss": {"fp32": 6.9, "stock": 7.0, "native": 6.95},
          "update_rel_vs_fp32": {"stock": 1.3, "native": 1.35},
          "fc_update_rel_vs_fp32": {"stock": 0.32, "native": 0.31}, "moved": {"native": 1.0}}
    assert selfcheck.check(ok) == []
    bad = dict(ok, update_rel_vs_fp32={"stock": 1.0, "native": 2.0})        # a wrong engine's update
    assert any("update_rel_vs_fp32" in b for b in selfcheck.check(bad))
    bad = dict(ok, loss={"fp32": 6.9, "stock": 7.0, "native": 8.0})
    assert any("native loss" in b for b in selfcheck.check(bad))
    bad = dict(ok, moved={"native": 0.0})
    assert any("did not move" in b for b in selfcheck.check(bad))
