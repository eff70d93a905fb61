"""tools/pmc_summary.py on synthetic rocprofv3 CSVs: per-kernel stats, the solo / overlapped
dispatch split bench.py's batches need, and the gfx950-corrected HBM bytes (2 x FETCH_SIZE +
WRITE_SIZE, both reported in KiB)."""

import csv
import importlib.util
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _load():
    spec = importlib.util.spec_from_file_location("pmc_summary", os.path.join(ROOT, "tools", "pmc_summary.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _write(path, header, rows):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(header)
        w.writerows(rows)


def test_summary_split_and_bytes(tmp_path):
    d = str(tmp_path)
    obs = "void nmmo::obs_kernel<false, false>(nmmo::ObsParams)"
    tick = "void nmmo::tick_kernel_w8<15u>(nmmo::DevState, int const*)"
    _write(os.path.join(d, "trace", "run_kernel_stats.csv"), ["Name", "Calls", "AverageNs"],
           [[obs, 4, 150.0], [tick, 2, 10.0]])
    # obs: [0,100) alone, [200,400) and [300,500) overlap each other, [600,700) alone
    _write(os.path.join(d, "trace", "run_kernel_trace.csv"), ["Kernel_Name", "Start_Timestamp", "End_Timestamp"],
           [[obs, 0, 100], [obs, 200, 400], [obs, 300, 500], [tick, 450, 460], [obs, 600, 700], [tick, 800, 810]])
    _write(os.path.join(d, "fetch", "run_counter_collection.csv"), ["Kernel_Name", "Counter_Name", "Counter_Value"],
           [[obs, "FETCH_SIZE", 10.0], [obs, "FETCH_SIZE", 30.0]])
    _write(os.path.join(d, "write", "run_counter_collection.csv"), ["Kernel_Name", "Counter_Name", "Counter_Value"],
           [[obs, "WRITE_SIZE", 100.0], [obs, "WRITE_SIZE", 100.0]])
    k = _load().summarise(d)
    o, t = k["obs_kernel"], k["tick_kernel"]  # the _w8 occupancy variant folds into its kernel
    assert o["dispatches"] == 4 and o["avg_ns"] == 150.0
    assert (o["solo_dispatches"], o["solo_avg_ns"]) == (2, 100.0)
    assert (o["overlapped_dispatches"], o["overlapped_avg_ns"]) == (2, 200.0)
    assert (t["solo_dispatches"], t["overlapped_dispatches"]) == (2, 0)
    assert o["hbm_bytes_per_dispatch"] == 2 * 20 * 1024 + 100 * 1024
    assert "hbm_bytes_per_dispatch" not in t
