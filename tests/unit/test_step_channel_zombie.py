"""A killed TP leader that its parent has not reaped (a zombie) counts as dead for the step
channel (csrc/runtime/proc.h pid_alive): a worker must not wait on it forever because its
launcher has not called wait() yet (the GPU dead-leader test raced on exactly that)."""
import os
import signal
import time
import uuid

from polykey_service_amd._native.loader import load_extension


def test_unreaped_dead_producer_is_not_alive():
    rt = load_extension("_pk_runtime")
    name = f"/pk_zombie_{uuid.uuid4().hex[:8]}"
    r, w = os.pipe()
    pid = os.fork()
    if pid == 0:  # the "leader": creates the channel as its producer, then waits to be killed
        try:
            os.close(r)
            ch = rt.StepChannel(name, True, 4, 1, 4096)  # noqa: F841 (kept alive until killed)
            os.write(w, b"x")
            time.sleep(60)
        finally:
            os._exit(0)
    os.close(w)
    try:
        assert os.read(r, 1) == b"x", "the producer process failed to create the channel"
        ch = rt.StepChannel(name, False, consumer_index=0)
        assert ch.producer_alive
        os.kill(pid, signal.SIGKILL)
        t0 = time.monotonic()
        while ch.producer_alive and time.monotonic() - t0 < 5:
            time.sleep(0.05)
        # not reaped yet (no waitpid so far): the child is a zombie, and the channel sees it dead
        assert not ch.producer_alive
        ch.close()
    finally:
        try:
            os.kill(pid, signal.SIGKILL)
        except ProcessLookupError:
            pass
        os.waitpid(pid, 0)
        try:
            os.unlink(f"/dev/shm{name}")
        except FileNotFoundError:
            pass
