"""The drop-in render() pass loop (bindings/rust/src/lib.rs `render`, restated
in massrt.render) against the reference's accounting (main.rs:150-295):
a frame = pre-pass, Image::clear, then workers x frame_limit whole 1-spp
passes (num_cpus - 2 render threads, main.rs:159-160, each rendering
frame_limit passes, main.rs:243-280), one merge (pass count + 1) per pass,
fresh samples every frame. CPU only: the image is a recorder.
"""
from __future__ import annotations

import os
import re

import pytest

import massrt
from conftest import REPO

LIB_RS = REPO / "bindings" / "rust" / "src" / "lib.rs"


class Recorder:
    """Stands in for massrt.Image: records the calls render() makes."""

    def __init__(self):
        self.calls = []
        self.passes = 0

    def prepass(self, seed):
        self.calls.append(("prepass", seed))

    def clear(self):
        self.calls.append(("clear",))
        self.passes = 0

    def render(self, seed, first, n, max_depth):
        self.calls.append(("render", seed, first, n, max_depth))
        self.passes += n


def renders(rec):
    return [c for c in rec.calls if c[0] == "render"]


def test_frame_has_workers_times_frame_limit_passes():
    rec, seen = Recorder(), []
    st = massrt.SampleStreams(7)
    done = massrt.render(rec, st, frame_limit=2, workers=5, batch=3, update=lambda im, p: seen.append(p))
    assert done == 10
    assert rec.calls[0] == ("prepass", 7) and rec.calls[1] == ("clear",)  # main.rs:162-233 order
    assert [(c[2], c[3]) for c in renders(rec)] == [(0, 3), (3, 3), (6, 3), (9, 1)]
    assert seen == [3, 6, 9, 10]  # Image::merge counts one pass per merged 1-spp pass
    assert all(c[1] == 7 and c[4] == massrt.MAX_DEPTH for c in renders(rec))


def test_frames_draw_fresh_samples():
    """Two render() calls (two animation frames, main.rs:104-120) never share
    a (seed, sample) pair, and each frame starts from a cleared image."""
    rec = Recorder()
    st = massrt.SampleStreams(1)
    massrt.render(rec, st, frame_limit=1, workers=4, batch=64)
    first = renders(rec)
    rec2 = Recorder()
    massrt.render(rec2, st, frame_limit=1, workers=4, batch=64)
    second = renders(rec2)
    s1 = {(c[1], c[2] + k) for c in first for k in range(c[3])}
    s2 = {(c[1], c[2] + k) for c in second for k in range(c[3])}
    assert len(s1) == len(s2) == 4 and not (s1 & s2)
    assert rec2.passes == 4  # not 8: the image was cleared (main.rs:233)


def test_unlimited_frame_stops_on_keep_going():
    """frame_limit None (the interactive case, main.rs:89-93): passes until
    QUICK_PASS; keep_going is consulted before every batch."""
    rec, checks = Recorder(), []

    def keep():
        checks.append(1)
        return len(checks) <= 3

    done = massrt.render(rec, massrt.SampleStreams(1), frame_limit=None, workers=3, batch=8, keep_going=keep)
    assert done == 24 and len(renders(rec)) == 3 and len(checks) == 4


def test_quick_pass_renders_nothing():
    rec = Recorder()
    done = massrt.render(rec, massrt.SampleStreams(1), frame_limit=3, workers=2, keep_going=lambda: False)
    assert done == 0 and renders(rec) == [] and rec.calls[0][0] == "prepass"


def test_seed_moves_on_before_sample_index_wraps():
    st = massrt.SampleStreams(5, next_sample=0xFFFFFFFF - 10)
    assert st.take(8) == (5, 0xFFFFFFFF - 10)
    assert st.take(8) == (6, 0)  # would have wrapped: next seed, samples from 0
    assert st.next_sample == 8


def test_default_workers_is_num_cpus_minus_two():
    assert massrt.default_workers() == max(1, (os.cpu_count() or 1) - 2)


def test_rust_render_states_the_same_loop():
    """lib.rs `render` is the loop restated above (no Rust toolchain here, so
    its statements are checked as text): pre-pass then clear, workers x
    frame_limit passes, batches of opts.batch, one update per batch,
    keep_going before each batch, SampleStreams::take for fresh samples."""
    src = LIB_RS.read_text()
    body = src[src.index("pub fn render<U, K>"):]
    order = ["image.prepass(streams.seed)", "image.clear()", "frame_limit.map(|f| f as u64 * opts.workers.max(1) as u64)",
             "if !keep_going()", "(t - done).min(batch)", "streams.take(k)", "image.render(seed, first, k, opts.max_depth)",
             "update(image, passes)"]
    pos = [body.index(s) for s in order]
    assert pos == sorted(pos)
    assert "(cpus - 2).max(1)" in src and "batch: 256" in src
    take = src[src.index("pub fn take(&mut self, n: u32)"):]
    assert re.search(r"self.next_sample as u64 \+ n as u64 > u32::MAX as u64", take)
    assert "render_passes" not in src  # the round-2 loop (frame_limit passes in total, fixed seed) is gone


@pytest.mark.parametrize("batch", [1, 7, 64])
def test_batching_does_not_change_the_sample_set(batch):
    rec = Recorder()
    massrt.render(rec, massrt.SampleStreams(3), frame_limit=3, workers=5, batch=batch)
    got = [c[2] + k for c in renders(rec) for k in range(c[3])]
    assert got == list(range(15))
