"""bench.py's measurement bookkeeping without a GPU: every workload names the
dominant kernel it times, the committed per-kernel PMC summary of that workload holds counters
of exactly that kernel (or the bench refuses it), and the flop models are the documented ones."""
import json
import math
import os

import pytest

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_workload_has_a_dominant_kernel():
    for tag in bench.PARAMS:
        fam, kname = bench.DOMINANT.get(tag, ("pbs_classic_kernel", bench.PARAMS[tag][2]))
        assert kname.split("<")[0] in bench.PARAMS[tag][2] or tag == "4_4", tag
        assert fam == kname.split("<")[0] or tag in ("mb3", "mb2"), tag


@pytest.mark.parametrize("tag", ["2_2", "2_2ks", "mb3", "mb2", "4_4", "3_3", "mb3_3g3"])
def test_committed_pmc_names_the_timed_kernel(tag):
    """profiles/r03_pmc_<tag>.json exists and has an entry for the kernel the bench times."""
    fam, kname = bench.DOMINANT[tag]
    e, why = bench.load_pmc(tag, kname)
    assert e is not None, why
    assert e["hbm_bytes_per_dispatch"] > 0
    assert 0 < e["valu_busy"] < 1


def test_pmc_of_another_kernel_is_refused(tmp_path, monkeypatch):
    prof = tmp_path / "profiles"
    prof.mkdir()
    (prof / f"{bench.PMC_ROUNDS[0]}_pmc_2_2.json").write_text(json.dumps(
        {"by_kernel": {"pbs_multibit_kernel<2048,1,1,3>": {"hbm_bytes_per_dispatch": 1.0}}}))
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    e, why = bench.load_pmc("2_2", "pbs_classic_kernel<2048,1,1>")
    assert e is None and "refused" in why


def test_pmc_entry_family_lookup():
    by = {"large_top_inv_kernel<32768,1,0>": {"x": 1}, "large_digits_kernel": {"x": 2}}
    assert bench.pmc_entry(by, "large_top_inv_kernel") == {"x": 1}   # timer family -> its one instantiation
    assert bench.pmc_entry(by, "large_digits_kernel") == {"x": 2}
    assert bench.pmc_entry(by, "large_group_cmux_kernel") is None


def test_flop_models():
    from tfhe_mi355.parameters import ALL

    p22 = ALL["PARAM_MESSAGE_2_CARRY_2_KS_PBS"]
    assert bench.pbs_flops(p22) == 194510848        # 262,144 flop per CMUX x 742
    p44 = ALL["PARAM_MESSAGE_4_CARRY_4_KS_PBS"]
    assert abs(bench.large_group_flops(p44) - 7667712) < 1
    p33 = ALL["PARAM_MESSAGE_3_CARRY_3_KS_PBS"]
    M = 4096
    assert bench.split_sub_flops(p33) == 2 * 2 * 5 * M * 10 + 4 * 2 * M * 8 + 2 * 5 * M * 10
    assert bench.split_dsub_flops(p33) == bench.split_sub_flops(p33) + 2 * 2 * (6 * M + 5 * M * math.log2(4))
    mb = ALL["PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS"]
    assert bench.split_sub_flops(mb) == bench.split_sub_flops(p33.with_(pbs_level=2)) + 7 * 4 * 2 * M * 8


def test_split_chunk_matches_the_engine_rule():
    """bench.split_chunk mirrors capi.cpp large_chunk: 200 MiB of (acc + spectra) per pass, a
    multiple of 64 in [64, 1024], 128 at N = 32768, 1024 for multi-bit."""
    from tfhe_mi355.parameters import ALL

    assert bench.split_chunk(ALL["PARAM_MESSAGE_3_CARRY_3_KS_PBS"], 4096) == 512
    assert bench.split_chunk(ALL["PARAM_MESSAGE_4_CARRY_4_KS_PBS"], 4096) == 128
    assert bench.split_chunk(ALL["PARAM_MESSAGE_1_CARRY_4_KS_PBS"], 4096) == 1024
    assert bench.split_chunk(ALL["PARAM_MESSAGE_2_CARRY_5_KS_PBS"], 4096) == 256
    assert bench.split_chunk(ALL["PARAM_MULTI_BIT_MESSAGE_3_CARRY_3_GROUP_3_KS_PBS"], 4096) == 1024


def test_mall_ceiling_is_the_committed_probe():
    txt = open(os.path.join(ROOT, "profiles", "r03_mall_stream_probe.log")).read()
    # working sets of 96-255 MiB: past the 32 MiB of L2, inside the 256 MiB Infinity Cache
    best = max(float(l.split(": ")[1].split(" TB/s")[0]) for l in txt.splitlines() if "TB/s" in l and "MiB x3" in l
               and 96 <= int(l.split("working set ")[1].split(" MiB")[0]) <= 255)
    assert abs(best * 1000 - bench.MALL_STREAM_GBS) < 50


def test_compact_summary_keeps_every_workload_and_the_callers():
    """The default line ends with a short per-workload summary (value, frac, one-call latency,
    64 / 256 blocking callers, mismatching rows) that a 2000-character tail of the output keeps."""
    sct = {"callers": {t: {"value": 1000.0 * int(t), "frac_of_batched_device_rate": 0.1, "mismatching_rows": 0,
                           "failed_calls": 0} for t in ("1", "64", "256")},
           "submit_wait": {"1x256": {"value": 7e4, "mismatching_rows": 0, "failed_calls": 0}}}
    head = {"value": 130000.0, "unit": "PBS/s", "ms_per_step": 31.5, "steps": 10, "n_gpus": 1,
            "config": {"workload": "w", "global_batch": 4096}, "roofline": {"frac": 0.318},
            "single_call_latency_ms": 2.5, "host_abi": {"single_ct": sct}}
    child = bench.summarize(dict(head, value=6000.0, host_abi={"single_ct": sct}))
    assert child["callers"]["callers_64"] == 64000.0 and child["callers"]["mismatching_rows"] == 0
    line = dict(head, other_workloads={"3_3": child, "4_4": {"error": "rc=1: boom", "wall_s": 1.0}})
    s = bench.compact_summary(line)
    assert s["2_2"] == {"v": 130000.0, "frac": 0.318, "lat_ms": 2.5, "c1": 1000.0, "c64": 64000.0,
                        "c256": 256000.0, "s1x256": 70000.0, "bad": 0}
    assert s["3_3"]["v"] == 6000.0 and s["3_3"]["c64"] == 64000.0
    assert "error" in s["4_4"]
    assert len(json.dumps(s)) < 1500
