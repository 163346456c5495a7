"""CPU: the trace / layout analysis tools behind the committed profiles (tools/kstats.py,
tools/kseq.py, tools/lds_bank_check.py) on synthetic inputs."""
import os
import sqlite3
import sys

import pytest

TOOLS = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools")
sys.path.insert(0, TOOLS)


@pytest.fixture
def trace_db(tmp_path):
    """A rocpd-like `kernels` table: two queues, each with a marker kernel bracketing two steps."""
    db = tmp_path / "t_results.db"
    c = sqlite3.connect(db)
    c.execute("create table kernels (name text, start int, end int, grid_x int, workgroup_x int, queue_id int)")
    rows = []
    for q in (1, 2):
        t = 1000 * q
        for step in range(3):
            for name, dur in (("void dv::conv_dma_kernel<0, 2>(dv::ConvArgs)", 10_000),
                              ("void dv::avgpool_fwd_kernel<0, 3>(...)", 5_000),
                              ("void dv::dream_update_kernel<0>(...)", 2_000)):
                rows.append((name, t, t + dur, 256 * 64, 256, q))
                t += dur + 1_000  # 1 us gap
    c.executemany("insert into kernels values (?, ?, ?, ?, ?, ?)", rows)
    c.commit()
    c.close()
    return str(db)


def test_kseq_one_step_per_queue(trace_db, capsys):
    import kseq

    kseq.main([trace_db, "--marker", "dream_update", "--nth", "0"])
    out = capsys.readouterr().out
    assert out.count("== queue") == 2
    assert "3 launches" in out  # conv, avgpool, dream_update between two markers
    assert "dv::conv_dma_kernel" in out and "idle gaps total 3.0 us" in out


def test_kstats_table(trace_db, capsys):
    import kstats

    kstats.main([trace_db, "--top", "5"])
    out = capsys.readouterr().out
    assert "dv::conv_dma_kernel<0, 2>" in out and "calls" in out


def test_lds_bank_check_layouts():
    from lds_bank_check import ways

    swz = lambda p: ((p >> 2) & 1) << 1  # noqa: E731  (KW3 / hs16 64-B rows)
    assert ways(lambda p, q: p * 64 + ((q ^ swz(p)) << 4)) == 1
    assert ways(lambda p, q: p * 160 + q * 16) == 1  # c64 halo pitch (round 3)
    assert ways(lambda p, q: p * 144 + q * 16) == 2  # the round-2 pitch
