"""Host-side logic of the product library (no GPU needed): symbol exports, parameter defaults,
the glibc rand() restatement and sample drawing.  CPU only."""
import re
import subprocess

import numpy as np

import clrrt
from clrrt import abi
from oracle_binding import Oracle, lib as olib


def _header_functions():
    txt = open(clrrt.HEADER_PATH).read()
    return sorted(set(re.findall(r"\b(clrrt_[a-z_0-9]+)\s*\(", txt)))


def test_library_loads_and_exports_every_header_symbol():
    L = clrrt.lib()
    assert L.clrrt_abi_version() == abi.CLRRT_ABI_VERSION == 11
    declared = _header_functions()
    assert len(declared) >= 25
    out = subprocess.run(["nm", "-D", "--defined-only", clrrt.LIB_PATH], capture_output=True, text=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [s for s in declared if s not in exported]
    assert not missing, missing
    assert set(clrrt.exported_symbols()) <= set(declared)


def test_abi_record_sizes_match_header():
    import ctypes as C
    assert C.sizeof(abi.Node) == 160
    assert C.sizeof(abi.Params) == 9 * 8 + 11 * 8 + 4 * 8 + 5 * 8 + 8 + 3 * 8 + 4 * 4
    assert C.sizeof(abi.SimCase) == 15 * 8 + 2 * 4  # clrrt_sim_case
    # clrrt_exchange_io (static_assert'ed 128 in clrrt_capi.hip): field offsets as the header lays them out
    io = abi.ExchangeIO
    assert C.sizeof(io) == 128
    assert [getattr(io, f).offset for f in ("elapsed_ms", "aux_local", "bbox_local", "stream", "dev_all", "n_all",
                                            "max_elapsed_ms", "aux_sum", "bbox_all")] == [8, 16, 24, 56, 64, 72, 80, 88, 96]


def test_params_default_matches_reference_values():
    p = clrrt.default_params()
    q = abi.default_params()
    assert bytes(p) == bytes(q)
    assert p.sim_dt == 0.04 and p.ctrl_Kp == 8 and p.Wcost[0] == 10 and p.ref_res == 0.2
    assert abs(p.veh.Kus - 0.013963) < 1e-6


def test_rng_matches_glibc_rand():
    for seed in (1, 2, 3, 42, 0, 2 ** 31 - 1):
        r = clrrt.Rng(seed)
        olib().orc_srand(seed)
        assert [r.next() for _ in range(2000)] == [olib().orc_rand() for _ in range(2000)]


def test_draw_samples_match_reference_sampling():
    for goal in ((40.0, 0.0, 0.0, 0.0), (30.0, 12.0, 0.3, 1.0)):
        p = clrrt.default_params(goal=goal)
        q = abi.default_params(goal=goal)
        r = clrrt.Rng(9)
        xy, ex = clrrt.samples_to_numpy(r.draw_samples(p, 500))
        o = Oracle(q)
        Oracle.srand(9)
        oxy, oex = o.draw_samples(500)
        assert np.array_equal(xy, oxy) and np.array_equal(ex, oex)
        assert 0.55 < ex.mean() < 0.85


def test_create_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        return
    try:
        clrrt.Planner(clrrt.default_params())
    except clrrt.ClrrtError:
        return
    raise AssertionError("Planner() must raise without a HIP device")


def test_bench_reads_committed_pmc_traffic():
    """bench.py's roofline.traffic comes from the newest committed FETCH_SIZE/WRITE_SIZE summaries of the
    benchmarked config;
    the kernel names carry template arguments that change between builds (k_roll_run<false, false>),
    so the reader must match every instantiation rather than one spelling."""
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("clrrt_bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    traffic, note = bench.measured_traffic("cfg3")
    assert traffic is not None, note
    assert 1e7 < traffic < 5e9, (traffic, note)
    # a config without committed PMC passes gets no traffic figure (not another config's)
    traffic, note = bench.measured_traffic("cfg_none")
    assert traffic is None and "no PMC profile" in note


def test_bench_cpu_share_is_bounded():
    import importlib.util
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    spec = importlib.util.spec_from_file_location("clrrt_bench", os.path.join(root, "bench.py"))
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    n = bench.cpu_share()
    assert 1 <= n <= (os.cpu_count() or 1)
