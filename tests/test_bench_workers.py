"""bench.run_workers (the PHY worker pool of the timed region) on CPU: every step is run exactly once over the
workers, each call's wall time is returned, the garbage collector is back on afterwards, and a worker's error reaches
the caller."""
import gc
import time

import pytest

import bench


class _Rx:
    def __init__(self, fail_at=None):
        self.batches, self.fail_at = [], fail_at

    def step(self, b):
        if self.fail_at is not None and len(self.batches) == self.fail_at:
            raise RuntimeError("worker failed")
        self.batches.append(b)
        time.sleep(0.0005)


@pytest.mark.parametrize("W,reps", [(1, 5), (3, 20), (3, 2)])
def test_steps_split_over_workers(W, reps):
    rxs = [_Rx() for _ in range(W)]
    calls = bench.run_workers(rxs, [[("b", w)] for w in range(W)], reps)
    assert len(calls) == reps and all(c > 0 for c in calls)
    assert [len(r.batches) for r in rxs] == [len(range(w, reps, W)) for w in range(W)]
    assert all(b == ("b", w) for w, r in enumerate(rxs) for b in r.batches)
    assert gc.isenabled()
    st = bench.call_stats(calls)
    assert st["calls"] == reps and 0 < st["p50_ms"] <= st["max_ms"]


def test_worker_error_reaches_caller():
    rxs = [_Rx(), _Rx(fail_at=1), _Rx()]
    with pytest.raises(RuntimeError, match="worker failed"):
        bench.run_workers(rxs, [[0], [0], [0]], 9)
    assert gc.isenabled()
    assert bench.call_stats([]) is None


def test_pool_threads_persist_across_runs():
    """warm-up and timed steps run on the same threads (a thread's first HIP calls carry one-off setup)"""
    import threading

    class _T(_Rx):
        def step(self, b):
            self.batches.append(threading.get_ident())

    rxs = [_T() for _ in range(3)]
    pool = bench.PhyWorkers(rxs)
    try:
        assert len(pool.run([[0]] * 3, 6)) == 6
        assert len(pool.run([[0]] * 3, 7)) == 7
    finally:
        pool.close()
    assert [len(r.batches) for r in rxs] == [2 + 3, 2 + 2, 2 + 2]
    assert all(len(set(r.batches)) == 1 for r in rxs)  # one thread per worker for both runs
    assert len({r.batches[0] for r in rxs}) == 3 and threading.get_ident() not in {r.batches[0] for r in rxs}
