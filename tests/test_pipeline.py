"""PipelinedReplay's host scheduling on the CPU (no GPU): three instances
coding one stream on their own threads, ordered by device events.  The
device is simulated: an event is "recorded" when its frame ends and a
stream wait checks that the event it waits on holds the frame it should
(a re-recorded ring slot would show up as a wrong frame).  Frames take
random times, the slow instance changes, and the run is long enough that
the 64-entry event ring wraps several times -- the round-5 bench hang (flags
dropped while a later frame could still wait on them) is what this pins."""
import random
import threading
import time

import pytest

from rav1e_amd import replay as RP


class _FakeLib:
    def __init__(self, slots=24):
        self.slots = slots  # rv_replay_dpb_slots
        self.lock = threading.Lock()
        self.events = {}   # handle -> the coded frame last recorded into it
        self.errors = []
        self._next = 1

    def rv_event_create(self):
        with self.lock:
            h = self._next
            self._next += 1
            self.events[h] = None
            return h

    def rv_event_destroy(self, h):
        return 0

    def rv_replay_dpb_slots(self):
        return self.slots

    def rv_event_record(self, ev, stream):
        with self.lock:
            self.events[ev] = stream.current
        return 0

    def rv_stream_wait_event(self, stream, ev):
        with self.lock:
            stream.waited.append(self.events[ev])
        return 0


class _Stream:
    def __init__(self):
        self.current = None
        self.waited = []


class _FakeInst:
    """What PipelinedReplay uses of a HipReplay instance."""

    def __init__(self, log, delay):
        self.cfg = type("Cfg", (), {"n_refs": 2})()
        self.stream = _Stream()
        self.log, self.delay = log, delay
        self.next = 0

    def seek(self, n):
        self.next = n

    def frame(self):
        n = self.next
        # every frame it depends on must have ended before it starts
        self.log.append(("start", n, list(self.stream.waited)))
        self.stream.waited = []
        time.sleep(self.delay(n))
        self.stream.current = n
        self.next += 1
        return {}

    def twin(self, stream=None):
        return _FakeInst(self.log, self.delay)

    def results(self):
        return []

    def close(self):
        pass


@pytest.mark.parametrize("seed,slots", [(1, 24), (2, 24), (3, 12)])
def test_pipelined_schedule_long_stream(monkeypatch, seed, slots):
    fake = _FakeLib(slots)
    monkeypatch.setattr(RP, "lib", lambda: fake)
    monkeypatch.setattr(RP, "_check", lambda rc, what: None)
    rnd = random.Random(seed)
    delays = {}

    def delay(n):
        # the level-1 / 4g+3 instances are slow in stretches
        j = (n - 1) % 4 if n else 0
        slow = (n // 40) % 3 == j % 3
        return delays.setdefault(n, rnd.uniform(0, 0.002) + (0.003 if slow else 0))
    log = []
    primary = _FakeInst(log, delay)
    p = RP.PipelinedReplay(primary)
    n_frames = 300
    done = threading.Event()

    def run():
        for _ in range(n_frames):
            p.frame()
        p.drain()
        done.set()
    t = threading.Thread(target=run, daemon=True)
    t.start()
    assert done.wait(120), "the pipeline deadlocked"
    # every coded frame ran once
    started = sorted(n for kind, n, _ in log if kind == "start")
    assert started == list(range(n_frames))
    # every wait a frame queued saw the event of the frame it depends on
    # (never a newer occupant of the ring slot)
    for kind, n, waited in log:
        deps = p._deps(n)
        assert sorted(waited) == sorted(deps), (n, waited, deps)
    # the flags of frames no later frame can wait on were dropped
    assert len(p.done) <= 3 * p.DEP_SPAN + 8
    p.close()
