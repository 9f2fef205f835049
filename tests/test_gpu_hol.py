"""A caller stream held up outside the library must not hold back another
thread's calls on another stream.

The reference's per-block callers are concurrent rayon workers
(src/vfs/mod.rs:91-97); a daemon may also hold a stream on a collective or a
host-released wait.  tools/hol_held.py holds stream A with
hipStreamWaitValue32 (released by the host after 1 s) behind library work
that uploads a new plan and takes upload-ring slots, while thread B runs
library calls on stream B that need the same plan and cycle every ring slot,
plus the submission queue and host-buffer calls (mapped and pageable) whose
scratch buffers grow during the hold -- grown without a free, since hipFree
waits for every stream of the device (r06 s40).  Since r06 the
library keeps a caller stream's readiness mirrors on a mirror stream of its
own, re-uploads a plan another stream still has in flight, and takes a ring
slot whose last reader has finished: none of B's steps may wait for A's
release -- unless the runtime itself holds B (B's plain torch kernel is the
baseline: streams share the GPU's hardware queues)."""
import pytest

pytestmark = pytest.mark.gpu


def test_held_stream_does_not_hold_back_others(gpu):
    from tools import hol_held
    r = hol_held.run(hold=1.0)
    assert "error" not in r and "error" not in r["b_steps_s"], r
    assert r["b_finished"], r
    if "torch_kernel_on_B" in r["b_steps_held_back"]:
        pytest.skip(f"the runtime holds stream B behind A (shared hardware queue): {r}")
    assert r["b_steps_held_back"] == [], r
