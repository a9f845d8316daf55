"""The kernel timer (phc_timer_*, KernelTimer): launches stamp their own start / end from the device's
constant-rate clock (phc_common.h launch_clock_begin / _end) — checked against HIP events around the
same launches, inside a captured hipGraph (where events cannot be timed on ROCm 7.2), and for the
reset / sampling bookkeeping bench.py relies on.  Needs an MI355X."""

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _gemm_operands(m=32768, n=1536, k=2048):
    g = torch.Generator(device=DEV).manual_seed(0)
    a = torch.randn((2, m, k), device=DEV, generator=g).half()
    b = (torch.randn((2, n, k), device=DEV, generator=g) / k ** 0.5).half()
    out = torch.empty((2, m, n), device=DEV, dtype=torch.float16)
    return a, b, out


def _launch(N, a, b, out):
    N.twin_gemm(a, b, N.EPI_STORE, out, (2, out.shape[2]))


def test_clock_matches_events_eager():
    """Per-launch time from the kernel's own stamps vs a stream event pair around each launch: the
    events also hold the dispatch overhead, so the stamps are a little shorter, never longer."""
    from puffer_phc_amd import _native as N

    a, b, out = _gemm_operands()
    for _ in range(3):
        _launch(N, a, b, out)
    torch.cuda.synchronize()
    t = N.KernelTimer(capacity=64)
    N.gemm_set_timer(t)
    try:
        evs = []
        for _ in range(8):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _launch(N, a, b, out)
            e1.record()
            evs.append((e0, e1))
        torch.cuda.synchronize()
        assert t.count == 8 and t.offered == 8
        flops = 2.0 * 32768 * 1536 * 2048 * 2
        assert t.work == pytest.approx(8 * flops)
        clock_ms = t.total_ms() / 8
        event_ms = sum(e0.elapsed_time(e1) for e0, e1 in evs) / 8
    finally:
        N.gemm_set_timer(None)
    assert 0.85 * event_ms <= clock_ms <= 1.02 * event_ms, (clock_ms, event_ms)


def test_graph_slots_hold_the_last_replay_and_reset():
    """Launches captured into a graph are stamped on every replay (the slot keeps the last one);
    reset() drops eager launches stamped before it but keeps graph slots a later replay re-stamps;
    a graph not replayed since the reset does not count."""
    from puffer_phc_amd import _native as N

    a, b, out = _gemm_operands(m=8192)
    _launch(N, a, b, out)
    torch.cuda.synchronize()
    t = N.KernelTimer(capacity=64, period=2)
    N.gemm_set_timer(t)
    try:
        for _ in range(4):  # eager: 2 of 4 stamped (period 2)
            _launch(N, a, b, out)
        torch.cuda.synchronize()
        assert t.count == 2
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        g = torch.cuda.CUDAGraph()
        with torch.cuda.stream(s), torch.cuda.graph(g):
            for _ in range(6):  # offered 6 more: 3 captured slots
                _launch(N, a, b, out)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        assert t.count == 2  # captured, not yet executed
        g.replay()
        torch.cuda.synchronize()
        assert t.count == 5
        t.reset()
        assert t.count == 0  # nothing ran since the reset
        N.gemm_set_timer(None)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(3):  # back to back: the slots hold the last replay
            g.replay()
        e1.record()
        torch.cuda.synchronize()
        assert t.count == 3
        per = t.total_ms() / 3
        graph_per = e0.elapsed_time(e1) / 18  # every launch of the three replays
    finally:
        N.gemm_set_timer(None)
    # the stamped launches are a sample of the replayed ones: within clock / DVFS noise of their mean
    assert 0.8 * graph_per < per <= 1.2 * graph_per, (per, graph_per)


def test_small_rollout_gemms_are_not_offered():
    """phc_twin_gemm launches of <= 4,096 rows (the rollout's) are not part of the timed family."""
    from puffer_phc_amd import _native as N

    a, b, out = _gemm_operands(m=4096, n=256, k=128)
    t = N.KernelTimer(capacity=8)
    N.gemm_set_timer(t)
    try:
        _launch(N, a, b, out)
        torch.cuda.synchronize()
        assert t.offered == 0 and t.count == 0
    finally:
        N.gemm_set_timer(None)
