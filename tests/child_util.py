"""Child-process plumbing for the GPU tests that run a check in its own process (a process group,
RCCL-in-graph state or tens of GB of tables stay out of the pytest process).

Child side: `child_main(main)` runs `main()`; on any exception it prints, to STDOUT and as its last
lines, the stage reached (`stage("...")` calls), `torch.cuda.mem_get_info()` and the traceback
between `__CHILD_FAIL__` markers, destroys the process group in `finally`, and exits 1.

Parent side: `run_child(argv, marker, timeout)` logs the parent's resident HBM before the spawn and,
on failure, asserts with the child's failure block FIRST in the message, so a driver that keeps only
the tail of the output still holds the traceback."""
import os
import subprocess
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_STAGE = ["start"]


def stage(name: str) -> None:
    _STAGE[0] = name
    print(f"[child stage] {name}", flush=True)


def _mem_line() -> str:
    try:
        import torch

        if torch.cuda.is_available() and torch.cuda.is_initialized():
            free, total = torch.cuda.mem_get_info()
            return (f"mem_get_info free {free / 2**30:.1f} GiB of {total / 2**30:.1f} GiB; this process reserved "
                    f"{torch.cuda.memory_reserved() / 2**30:.1f} GiB, allocated {torch.cuda.memory_allocated() / 2**30:.1f} GiB")
    except Exception as e:  # noqa: BLE001 - diagnostics must not raise
        return f"mem_get_info unavailable: {e!r}"
    return "cuda not initialised"


def child_main(main) -> None:
    rc = 1
    try:
        rc = main() or 0
    except BaseException:  # noqa: BLE001 - report everything, including SystemExit from asserts
        tb = traceback.format_exc()
        print("__CHILD_FAIL__", flush=True)
        print(f"stage: {_STAGE[0]}", flush=True)
        print(_mem_line(), flush=True)
        print(tb, flush=True)
        print("__CHILD_FAIL_END__", flush=True)
        rc = 1
    finally:
        try:
            import torch.distributed as dist

            if dist.is_available() and dist.is_initialized():
                dist.destroy_process_group()
        except Exception:  # noqa: BLE001
            pass
    sys.stdout.flush()
    sys.exit(rc)


def seed_all(default: int) -> int:
    """Seed torch's global generators (model init: table uniform_, nn.Linear) from TT_TEST_SEED or
    `default`, so a child's run is reproducible; returns the seed (printed by the child)."""
    import torch

    seed = int(os.environ.get("TT_TEST_SEED", default))
    torch.manual_seed(seed)
    print(f"[child seed] {seed}", flush=True)
    return seed


def margin(got, want, rtol: float, atol: float) -> float:
    """max |got - want| / (atol + rtol |want|): <= 1 is what np.testing.assert_allclose accepts."""
    import numpy as np

    got, want = np.asarray(got, np.float64), np.asarray(want, np.float64)
    if got.size == 0:
        return 0.0
    return float(np.max(np.abs(got - want) / (atol + rtol * np.abs(want))))


def parent_mem() -> str:
    return "parent: " + _mem_line()


def failure_message(rc, out: str, err: str) -> str:
    """The child's failure block first, then short tails of its stdout / stderr."""
    block = ""
    if "__CHILD_FAIL__" in out:
        block = out[out.rindex("__CHILD_FAIL__"):]
        block = block[:block.find("__CHILD_FAIL_END__")] if "__CHILD_FAIL_END__" in block else block
        # keep the traceback's end (the raising frame and the message): the driver keeps tails
        block = block[-6000:]
    return f"child rc={rc}\n{block}\n--- stdout tail ---\n{out[-1500:]}\n--- stderr tail ---\n{err[-1500:]}"


def run_child(argv, marker: str, timeout: int, env=None):
    """Run `python argv...` from the repo root; assert rc 0 and `marker` in its stdout."""
    before = parent_mem()
    print(before, flush=True)
    r = subprocess.run([sys.executable, *argv], capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)
    if not (r.returncode == 0 and marker in r.stdout):
        import pytest

        msg = failure_message(r.returncode, r.stdout, r.stderr) + "\n" + before
        # pytest.fail prints the message untruncated (an `assert x, msg` explanation is cut to 8
        # lines); the captured-stdout copy lands at the very end of the report
        print(msg, flush=True)
        pytest.fail(msg, pytrace=False)
    return r
