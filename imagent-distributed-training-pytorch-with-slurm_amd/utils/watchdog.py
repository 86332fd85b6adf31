"""Hang watchdog with recovery by exit.

The reference has no failure detection beyond the Slurm wall limit
(``imagenet.sh:12``, 144 h) and NCCL's own timeout: a dead peer leaves every
other rank blocked in a collective until then. Here the training loop beats a
heartbeat every step; if no beat arrives for ``timeout`` seconds the watchdog
thread

1. dumps every thread's Python stack to stderr (where it hung),
2. aborts the communicators (``ncclCommAbort`` on our RCCL communicator, the
   c10d group abort) so no collective keeps the GPU queue blocked,
3. exits the process with a non-zero status (``os._exit``; never exec), so
   ``torchrun`` / ``srun`` tears down the job instead of it idling for days.

Fault injection for tests: ``IMAGENT_FAULT_STALL=<rank>:<step>:<seconds>``
makes that rank sleep before that training step (:func:`maybe_stall`);
``IMAGENT_FAULT_SLOW_SAVE=<seconds>`` makes the master's end-of-epoch checkpoint
write take that much longer (:func:`slow_save`).
"""

from __future__ import annotations

import faulthandler
import os
import sys
import threading
import time
from typing import Callable, List, Optional

EXIT_CODE = 75  # EX_TEMPFAIL: the job may be retried / resumed from its checkpoint


class Watchdog:
    def __init__(self, timeout: float, aborts: Optional[List[Callable[[], None]]] = None,
                 label: str = "", exit_code: int = EXIT_CODE, poll: Optional[float] = None):
        self.timeout = float(timeout)
        self.aborts = list(aborts or [])
        self.label = label
        self.exit_code = exit_code
        self._armed = False
        self._last = time.monotonic()
        self._what = ""
        self._stop = threading.Event()
        self._poll = poll if poll is not None else max(0.05, min(1.0, self.timeout / 10))
        self._thread = threading.Thread(target=self._run, name="imagent-watchdog", daemon=True)
        if self.timeout > 0:
            self._thread.start()

    def beat(self, what: str = "") -> None:
        """Heartbeat: the loop made progress (also arms the watchdog)."""
        self._last = time.monotonic()
        self._what = what
        self._armed = True

    def pause(self) -> None:
        """Disarm (e.g. while writing a checkpoint); the next beat re-arms."""
        self._armed = False

    def close(self) -> None:
        self._armed = False
        self._stop.set()

    def _run(self) -> None:
        while not self._stop.wait(self._poll):
            if self._armed and time.monotonic() - self._last > self.timeout:
                self._fire()
                return

    def _fire(self) -> None:
        msg = (f"[watchdog{(' ' + self.label) if self.label else ''}] no progress for {self.timeout:.0f} s "
               f"(last: {self._what or 'start'}); dumping stacks, aborting communicators, exiting "
               f"with status {self.exit_code}")
        try:
            print(msg, file=sys.stderr, flush=True)
            faulthandler.dump_traceback(file=sys.stderr, all_threads=True)
        except Exception:
            pass
        for fn in self.aborts:
            try:
                fn()
            except Exception as e:  # keep going: the exit is what matters
                print(f"[watchdog] abort hook failed: {e}", file=sys.stderr, flush=True)
        sys.stderr.flush()
        sys.stdout.flush()
        os._exit(self.exit_code)


def maybe_stall(rank: int, step: int) -> None:
    spec = os.environ.get("IMAGENT_FAULT_STALL")
    if not spec:
        return
    r, s, secs = spec.split(":")
    if int(r) == rank and int(s) == step:
        print(f"[fault injection] rank {rank} stalls {secs} s before step {step}", file=sys.stderr, flush=True)
        time.sleep(float(secs))


def slow_save() -> None:
    secs = os.environ.get("IMAGENT_FAULT_SLOW_SAVE")
    if secs:
        print(f"[fault injection] checkpoint write stalls {secs} s", file=sys.stderr, flush=True)
        time.sleep(float(secs))
