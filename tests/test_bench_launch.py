"""bench.py's own rank launcher (``--gpus N`` without torch.distributed.run) and the configs[3]
strong-scaling run with the host-side ordered merge (bench.strong_scaling, shard.SharedResults).

CPU: the launcher must fail non-zero when its ranks cannot run (no GPU here) instead of quietly
measuring one rank.  GPU: two ranks sharing cuda:0 scan one pair stream round-robin through the
real kernel, merge the results in input order and must equal the single-rank scan byte for byte.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env():
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return env


def test_launcher_fails_when_ranks_fail():
    import torch
    if torch.cuda.is_available():
        pytest.skip("checks the failure path on a host without GPUs")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--warmup", "1", "--no-cpu-baseline", "--no-extra"], env=_env(), cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "failed" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


@pytest.mark.gpu
def test_two_ranks_strong_scaling_merge_equals_single_rank():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "cdr1as",
                        "--pairs", "1000000", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-extra"],
                       env=_env(), cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2
    st = line["strong_scaling"]
    assert st["ranks"] == 2 and st["pairs_total"] == 1_000_000
    assert st["merged_equals_single_rank"] is True
    assert st["value"] > 0 and line["value"] > 0


def _bench(gpus, extra):
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--gpus", str(gpus), "--workload", "hg19",
                        "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-extra"] + extra,
                       env=_env(), cwd=ROOT, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


@pytest.mark.gpu
def test_two_ranks_configs3_and_configs4_on_hg19():
    """configs[3] and configs[4] on their own workload (hg19-shaped genome) through the real kernel with
    two ranks (both on the box's GPU; an 8-GPU node runs the same code with one GPU each):
    configs[3] -- an 8M-pair stream dealt round-robin, each rank generating only its batches, merged in
    the 2- and 4-byte forms -- equals the single-rank scan word for word; configs[4] -- an 8M-pair 120-150 bp
    stream in two contiguous shares -- has the same order-sensitive results checksum as one rank."""
    extra = ["--pairs", "8000000", "--config4-pairs", "8000000"]
    one = _bench(1, extra)
    two = _bench(2, extra)
    for line, ranks in ((one, 1), (two, 2)):
        st = line["strong_scaling"]
        assert line["n_gpus"] == ranks and st["ranks"] == ranks and st["pairs_total"] == 8_000_000
        assert st["merged_equals_single_rank"] is True
        assert st["merge_bytes_per_pair"] == 2 and st["merge_4B_words"]["merged_equals_single_rank"] is True
        assert st["merge_2B_copied"]["merged_equals_single_rank"] is True
        c4 = line["configs4_200M_150bp"]
        assert c4["ranks"] == ranks and c4["pairs_total"] == 8_000_000
    assert one["configs4_200M_150bp"]["results_checksum"] == two["configs4_200M_150bp"]["results_checksum"]
    assert two["configs4_200M_150bp"]["pairs_per_rank"] == 4_000_000


@pytest.mark.gpu
@pytest.mark.timeout(1200)
def test_two_ranks_full_size_configs3_and_configs4():
    """The driver's N = 2 launch at the full sizes, so that the 8-GPU SCALE run exercises nothing
    untested: configs[3]'s whole 50M-pair stream dealt round-robin to two ranks and merged through
    the zero-copy 2-byte form equals the single-rank scan word for word (and the 4-byte and copied
    forms too); configs[4]'s 200M-pair 120-150 bp stream in two shares has the single-rank
    order-sensitive results checksum.  Per-rank shared-memory and page-locked sizes are those of
    the N = 8 run."""
    one = _bench(1, ["--no-cli"])
    two = _bench(2, ["--no-cli"])
    for line, ranks in ((one, 1), (two, 2)):
        st = line["strong_scaling"]
        assert line["n_gpus"] == ranks and st["ranks"] == ranks and st["pairs_total"] == 50_000_000
        assert st["merged_equals_single_rank"] is True
        assert st["merge_4B_words"]["merged_equals_single_rank"] is True
        assert st["merge_2B_copied"]["merged_equals_single_rank"] is True
        assert st["merge_ms_per_step"] > -0.5                  # the host destination's cost, not a kernel swap
        c4 = line["configs4_200M_150bp"]
        assert c4["ranks"] == ranks and c4["pairs_total"] == 200_000_000
    assert one["configs4_200M_150bp"]["results_checksum"] == two["configs4_200M_150bp"]["results_checksum"]
