"""CPU: bench.py's algorithmic-byte accounting against the
figures the GPU runs reported (profiles/r01/methods/, whose PMC traffic
matched them within 0.1%)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

HEADLINE = [(4096, 4096, 1), (2048, 2048, 1), (1024, 1024, 1), (512, 512, 1), (256, 256, 1)]
VOLUME = [(1024, 1024, 256), (512, 512, 128), (256, 256, 64)]


@pytest.mark.parametrize("method,read,total", [
    ("mean", 2147483648, 2860515328),
    ("min", 2147483648, 2860515328),
    ("decimate", 1073741824, 1786773504),   # even rows only
])
def test_headline_bytes(method, read, total):
    counts = [0, 64, 64, 64, 64]
    assert bench.algorithmic_bytes(HEADLINE, counts, 64, method, 2) == (read, total)
    # 44,695,552 B per Mean frame
    if method == "mean":
        assert total // 64 == 44695552


@pytest.mark.parametrize("method,read,total", [
    ("mean", 536870912, 612368384),
    ("decimate", 134217728, 209715200),     # even planes, even rows
])
def test_volume_bytes(method, read, total):
    counts = [0, 128, 64]
    assert bench.algorithmic_bytes(VOLUME, counts, 256, method, 2) == (read, total)


def test_decimate_z_only_level_reads_every_row():
    # level 1 halves Z only: Decimate needs every row of the even planes
    geo = [(64, 48, 8), (64, 48, 4)]
    read, total = bench.algorithmic_bytes(geo, [0, 4], 8, "decimate", 1)
    assert read == 4 * 48 * 64
    assert total == read + 4 * 48 * 64


def test_odd_height_decimate_rows():
    geo = [(10, 7, 1), (5, 4, 1)]
    read, _ = bench.algorithmic_bytes(geo, [0, 3], 3, "decimate", 4)
    assert read == 3 * 4 * 10 * 4


# ---- --gpus N: the launcher ------------------------------

def test_gpus_without_launcher_starts_n_ranks():
    args = bench.parse(["--gpus", "8", "--steps", "3"])
    assert bench.resolve_world(args, {}) == ("launch", 8)
    cmd = bench.launcher_cmd(["--gpus", "8", "--steps", "3"], 8, 29555)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29555" in cmd
    i = cmd.index(os.path.abspath(bench.__file__))
    assert cmd[i + 1:] == ["--gpus", "8", "--steps", "3"]  # same arguments


def test_single_gpu_runs_in_process():
    assert bench.resolve_world(bench.parse([]), {}) == ("run", 1)
    assert bench.resolve_world(bench.parse(["--gpus", "1"]), {}) == ("run", 1)


def test_under_launcher_world_size_wins():
    # the driver: torch.distributed.run --nproc-per-node N bench.py --gpus N
    env = {"WORLD_SIZE": "4", "RANK": "2"}
    assert bench.resolve_world(bench.parse(["--gpus", "4"]), env) == ("run", 4)
    assert bench.resolve_world(bench.parse([]), env) == ("run", 4)
    with pytest.raises(SystemExit):
        bench.resolve_world(bench.parse(["--gpus", "8"]), env)


def test_aux_leg_reports_a_failure_in_the_line(capsys):
    # an auxiliary e2e leg that raises leaves {"error": ...} in the line (and
    # its traceback on stderr) instead of losing the line or stranding ranks
    assert bench.aux_leg("ok", lambda a, b=0: {"v": a + b}, 1, b=2) == {"v": 3}

    def boom():
        raise RuntimeError("hipErrorPeerAccessUnsupported")
    out = bench.aux_leg("e2e.node", boom)
    assert out == {"error": "RuntimeError: hipErrorPeerAccessUnsupported"}
    assert "e2e.node failed" in capsys.readouterr().err


def test_rotation_copies_keep_small_read_sets_out_of_the_cache():
    """Launch buffer sets (bench.rotation_copies): reads summed over the sets
    reach the target, so a launch never finds its input in the 256 MB
    Infinity Cache; batches that read >= the target keep one set."""
    import bench
    mib = 1 << 20
    # headline: 64 x 32 MiB frames, Mean reads all 2 GiB
    assert bench.rotation_copies(2048 * mib, "mean", False, 1024) == 1
    assert bench.rotation_copies(2048 * mib, "decimate", False, 1024) == 1
    # config V: one 512 MiB volume; Decimate reads every other row and plane
    assert bench.rotation_copies(512 * mib, "mean", True, 1024) == 2
    assert bench.rotation_copies(512 * mib, "decimate", True, 1024) == 8
    # config C1b: 1024 x 512^2 u8 = 256 MiB, Decimate reads half the rows
    assert bench.rotation_copies(256 * mib, "max", False, 1024) == 4
    assert bench.rotation_copies(256 * mib, "decimate", False, 1024) == 8
    # off, and the cap
    assert bench.rotation_copies(512 * mib, "decimate", True, 0) == 1
    assert bench.rotation_copies(mib, "mean", False, 1024) == 64
