"""Source stamps of the committed profiles (zkgpu/stamp.py) and bench.py's
choice of the profile a figure comes from: the newest profile whose stamp
matches the current sources of the kernel family it prices, stale otherwise.
CPU only."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "zkevm-prover_amd")]


def test_stamp_depends_on_sources_and_env(tmp_path, monkeypatch):
    from zkgpu import stamp
    s0 = stamp.all_stamps()
    assert set(s0) == {"lde", "poseidon", "zxp"} and all(len(v) == 16 for v in s0.values())
    # a build setting of a family changes only that family's stamp
    env = dict(os.environ, ZKGPU_LDE3="1")
    s1 = stamp.all_stamps(env)
    assert s1["lde"] != s0["lde"] and s1["poseidon"] == s0["poseidon"] and s1["zxp"] == s0["zxp"]
    env = dict(os.environ, ZKGPU_ZXP_MAX_TERMS="16")
    s2 = stamp.all_stamps(env)
    assert s2["zxp"] != s0["zxp"] and s2["lde"] == s0["lde"]
    # every environment setting the native code still reads is either listed
    # here or not a kernel setting
    import re
    src = ""
    for d in ("csrc", "host"):
        for fn in os.listdir(os.path.join(stamp.PKG, d)):
            src += open(os.path.join(stamp.PKG, d, fn), errors="replace").read()
    read = set(re.findall(r'getenv\("(ZKGPU_\w+)"\)', src))
    not_kernel = {"ZKGPU_ZXP_JIT", "ZKGPU_JIT_CACHE", "ZKGPU_JIT_LOG", "ZKGPU_ZXP_JIT_THREADS", "ZKGPU_ZXP_JIT_ONLY",
                  "ZKGPU_ZXP_JIT_DUMP", "ZKGPU_RUN_ID", "ZKGPU_COMM_TIMEOUT_S", "ZKGPU_LEAN_KEEP_COLS",
                  "ZKGPU_SYNC_STAGES", "ZKGPU_TEST_FAIL_EXCHANGE"}
    listed = {k for v in stamp.ENV.values() for k in v}
    assert read <= listed | not_kernel, read - listed - not_kernel
    # the interpreter/compiled switch is not a kernel setting
    assert stamp.all_stamps(dict(os.environ, ZKGPU_ZXP_JIT="0"))["zxp"] == s0["zxp"]
    ok, why = stamp.check({"stamps": s0}, "zxp")
    assert ok, why
    ok, why = stamp.check({"stamps": dict(s0, zxp="0" * 16)}, "zxp")
    assert not ok and "!=" in why
    ok, why = stamp.check({}, "lde")
    assert not ok and "no source stamp" in why


def test_bench_picks_newest_matching_profile(tmp_path, monkeypatch):
    """A newer-named but stale profile does not shadow an older matching one
    (r04a_* sorts after r04_*); with no match the newest is reported stale."""
    import bench
    from zkgpu import stamp
    prof = tmp_path / "profiles"
    prof.mkdir()
    cur = stamp.all_stamps()
    (prof / "r04_x_pmc.json").write_text(json.dumps({"stamps": cur, "v": "current"}))
    (prof / "r04a_x_pmc.json").write_text(json.dumps({"stamps": dict(cur, zxp="f" * 16), "v": "stale"}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    f, d, why = bench._stamped("*_x_pmc.json", "zxp")
    assert d is not None and d["v"] == "current" and f.endswith("r04_x_pmc.json")
    # the stale one is still fine for a family whose sources it matches
    f, d, why = bench._stamped("*_x_pmc.json", "lde")
    assert d["v"] == "stale" and f.endswith("r04a_x_pmc.json")
    (prof / "r04_x_pmc.json").unlink()
    f, d, why = bench._stamped("*_x_pmc.json", "zxp")
    assert d is None and why.startswith("stale") and f.endswith("r04a_x_pmc.json")
    f, d, why = bench._stamped("*_nothing.json", "zxp")
    assert f is None and d is None and "no committed" in why

