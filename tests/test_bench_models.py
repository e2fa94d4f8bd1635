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
    multiple of 64 in [64, 1024], 128 at N = 32768."""
    from tfhe_mi355.parameters import ALL

    assert bench.split_chunk(ALL["PARAM_MESSAGE_3_CARRY_3_KS_PBS"], 4096) == 512
    assert bench.split_chunk(ALL["PARAM_MESSAGE_4_CARRY_4_KS_PBS"], 4096) == 128
    assert bench.split_chunk(ALL["PARAM_MESSAGE_1_CARRY_4_KS_PBS"], 4096) == 1024
    assert bench.split_chunk(ALL["PARAM_MESSAGE_2_CARRY_5_KS_PBS"], 4096) == 256


def test_mall_ceiling_is_the_committed_probe():
    txt = open(os.path.join(ROOT, "profiles", "r03_mall_stream_probe.log")).read()
    # working sets of 96-255 MiB: past the 32 MiB of L2, inside the 256 MiB Infinity Cache
    best = max(float(l.split(": ")[1].split(" TB/s")[0]) for l in txt.splitlines() if "TB/s" in l and "MiB x3" in l
               and 96 <= int(l.split("working set ")[1].split(" MiB")[0]) <= 255)
    assert abs(best * 1000 - bench.MALL_STREAM_GBS) < 50
