"""Supervised benchmark runs: the timed job runs in a child process per rank, and a failed attempt
is retried ONCE per fallback path by fresh children, so one failure never loses the number.

The reference has no multi-GPU path; its per-GPU step (knearests.cu:235-392) is what
the scaling run repeats on every rank. Our N-GPU timed path is the native RCCL pipeline
(csrc/runtime/dist.cpp). A crash, a CollectiveError, a deadline abort or a missing JSON line on ANY
rank fails the attempt on EVERY rank:

* Each torchrun worker (a *parent*) never touches the GPU: it starts one child with the same
  RANK / WORLD_SIZE / LOCAL_RANK and a fresh rendezvous port, streams the child's stderr through,
  and keeps the child's stdout (rank 0's holds the JSON line).
* The parents coordinate over a TCP key-value store (torchrun's agent store, or one rank 0
  hosts): a failed child increments ``fail``, a finished one ``done``. When ``fail`` > 0 every
  parent kills its child's process group (exact pgid, never a pattern), waits until all children
  are gone, and the next attempt starts with its own environment (e.g. ``KN_DIST_PIPE=0``: the
  torch steady path) on a new port.
* Rank 0's parent prints the successful attempt's JSON line with ``dist_path`` (the attempt that
  produced it), ``first_attempt_rc`` and the failed attempts' last stderr lines.

Processes are started with ``subprocess`` (never ``exec``), so no process that initialised the GPU
is ever replaced.
"""
from __future__ import annotations

import collections
import json
import os
import signal
import socket
import subprocess
import sys
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Optional


@dataclass
class Attempt:
    name: str
    env: dict = field(default_factory=dict)     # environment overrides of the child
    argv: list = field(default_factory=list)    # extra command-line arguments of the child
    timeout_s: float = 300.0


@dataclass
class Outcome:
    rc: int
    line: Optional[dict]
    stderr_tail: list
    first_failure: Optional[dict] = None   # {"rank", "rc", "stderr_tail"} of the rank that failed first
    rcs: Optional[list] = None             # every rank's exit code (rank 0 only; None: unknown)
    failures: Optional[list] = None        # every failing rank's {"rank", "rc", "stderr_tail"} (rank 0)


def free_port(host: str = "127.0.0.1") -> int:
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind((host, 0))
    port = s.getsockname()[1]
    s.close()
    return port


def json_line(text: str) -> Optional[dict]:
    """The last stdout line that parses as a JSON object with a ``metric`` key."""
    for ln in reversed(text.splitlines()):
        ln = ln.strip()
        if ln.startswith("{"):
            try:
                d = json.loads(ln)
            except ValueError:
                continue
            if isinstance(d, dict) and "metric" in d:
                return d
    return None


class _Child:
    """One child process in its own process group; stderr streamed through (last lines kept),
    stdout collected."""

    def __init__(self, cmd: list, env: dict, tail: int = 30):
        self.p = subprocess.Popen(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                  start_new_session=True)
        self.out: list = []
        self.err = collections.deque(maxlen=tail)
        self._t = [threading.Thread(target=self._pump_out, daemon=True),
                   threading.Thread(target=self._pump_err, daemon=True)]
        for t in self._t:
            t.start()

    def _pump_out(self):
        for b in iter(self.p.stdout.readline, b""):
            self.out.append(b.decode(errors="replace"))

    def _pump_err(self):
        for b in iter(self.p.stderr.readline, b""):
            s = b.decode(errors="replace")
            self.err.append(s.rstrip("\n"))
            sys.stderr.write(s)
            sys.stderr.flush()

    def poll(self) -> Optional[int]:
        return self.p.poll()

    def kill(self) -> int:
        if self.p.poll() is None:
            try:
                os.killpg(self.p.pid, signal.SIGKILL)  # the group this child leads (start_new_session)
            except ProcessLookupError:
                pass
        rc = self.p.wait()
        for t in self._t:
            t.join(timeout=5)
        return rc

    def finish(self) -> Outcome:
        rc = self.kill()
        return Outcome(rc, json_line("".join(self.out)), list(self.err))


class _Coord:
    """Cross-rank counters for one attempt (a TCP store); a world of one needs none."""

    def __init__(self, rank: int, world: int, store=None):
        self.rank, self.world, self.store = rank, world, store
        self.local: dict = {}

    def add(self, key: str, v: int) -> int:
        if self.store is not None:
            return int(self.store.add(key, v))
        self.local[key] = int(self.local.get(key, 0)) + v
        return self.local[key]

    def set(self, key: str, v: str) -> None:
        if self.store is not None:
            self.store.set(key, v)
        else:
            self.local[key] = v

    def get(self, key: str) -> Optional[str]:
        if self.store is not None:
            if not self.store.check([key]):
                return None
            return self.store.get(key).decode()
        return self.local.get(key)

    def value(self, key: str) -> int:
        return self.add(key, 0)

    def barrier(self, key: str, timeout_s: float = 120.0) -> None:
        if self.store is None:
            return
        self.add(key, 1)
        t0 = time.monotonic()
        while self.value(key) < self.world:
            if time.monotonic() - t0 > timeout_s:
                raise TimeoutError(f"supervisor barrier {key}")
            time.sleep(0.1)

    def leave(self, key: str, timeout_s: float = 60.0) -> None:
        """Last store operation of every rank: rank 0 (which may host the store) waits until all
        ranks made theirs, the others return at once."""
        if self.store is None:
            return
        self.add(key, 1)
        t0 = time.monotonic()
        while self.rank == 0 and self.value(key) < self.world and time.monotonic() - t0 < timeout_s:
            time.sleep(0.05)

    def share(self, key: str, make: Callable[[], str]) -> str:
        if self.store is None:
            return make()
        if self.rank == 0:
            v = make()
            self.store.set(key, v)
            return v
        return self.store.get(key).decode()


def make_store(rank: int, world: int):
    """Parent-side store: torchrun's agent store (TORCHELASTIC_USE_AGENT_STORE=True) or one that
    rank 0 hosts on MASTER_PORT; keys under a per-run prefix."""
    if world <= 1:
        return None
    from datetime import timedelta

    import torch.distributed as dist

    host = os.environ.get("MASTER_ADDR", "127.0.0.1")
    port = int(os.environ.get("MASTER_PORT", "29500"))
    agent = os.environ.get("TORCHELASTIC_USE_AGENT_STORE") == "True"
    st = dist.TCPStore(host, port, None if agent else world, (rank == 0) and not agent,
                       timedelta(seconds=600), wait_for_workers=False)
    run = os.environ.get("TORCHELASTIC_RUN_ID", "none") + "/" + os.environ.get("TORCHELASTIC_RESTART_COUNT", "0")
    return dist.PrefixStore(f"kn_bench_supervisor/{run}/", st)


def supervise(cmd: list, attempts: list, rank: int = 0, world: int = 1, store=None,
              poll_s: float = 0.2) -> tuple:
    """Run ``cmd`` as this rank's child once per attempt until an attempt succeeds on every rank.
    Returns (index of the successful attempt or -1, [Outcome of this rank per attempt])."""
    co = _Coord(rank, world, store)
    outcomes = []
    for i, a in enumerate(attempts):
        port = int(co.share(f"a{i}/port", lambda: str(free_port())))
        env = dict(os.environ)
        env.update({"KN_BENCH_CHILD": "1", "MASTER_ADDR": env.get("MASTER_ADDR", "127.0.0.1"),
                    "MASTER_PORT": str(port), "TORCHELASTIC_USE_AGENT_STORE": "False"})
        env.update({k: str(v) for k, v in a.env.items()})
        child = _Child(list(cmd) + list(a.argv), env)
        t0 = time.monotonic()
        reported = False
        failed = False

        def report_failure(rc_desc):
            # every failing rank leaves its exit code and last stderr lines for rank 0's JSON line
            # (written BEFORE fail is raised, so a rank that sees fail > 0 and passes the exit barrier
            # finds them); fail before done, so done == world implies fail is final. The first to
            # fail is not always the cause: a peer blocked in a collective may die first
            rec = {"rank": rank, "rc": rc_desc, "stderr_tail": list(child.err)[-12:]}
            co.set(f"a{i}/failrec/{rank}", json.dumps(rec))
            if co.add(f"a{i}/fail", 1) == 1:
                co.set(f"a{i}/first", json.dumps(rec))

        while True:
            rc = child.poll()
            if rc is not None and not reported:
                reported = True
                ok = rc == 0
                if ok and rank == 0:
                    # rank 0's child must have printed the line (its pump may lag the exit)
                    child.kill()
                    ok = json_line("".join(child.out)) is not None
                if not ok:
                    report_failure(rc if rc != 0 else "no JSON line")
                co.add(f"a{i}/done", 1)
            if not reported and time.monotonic() - t0 > a.timeout_s:
                sys.stderr.write(f"[supervisor rank {rank}] attempt {a.name}: no exit within {a.timeout_s:.0f} s\n")
                report_failure(f"timeout {a.timeout_s:.0f} s")
                reported = True
                co.add(f"a{i}/done", 1)
            if co.value(f"a{i}/fail") > 0:
                failed = True
                break
            if co.value(f"a{i}/done") >= world:
                failed = co.value(f"a{i}/fail") > 0
                break
            time.sleep(poll_s)
        out = child.finish()
        outcomes.append(out)
        if not failed:
            co.leave("end")
            return i, outcomes
        sys.stderr.write(f"[supervisor rank {rank}] attempt {a.name} failed (rc {out.rc}); "
                         + (f"next: {attempts[i + 1].name}\n" if i + 1 < len(attempts) else "no attempts left\n"))
        co.set(f"a{i}/rc/{rank}", str(out.rc))
        co.barrier(f"a{i}/exited")  # every child of this attempt is gone before the next starts
        first = co.get(f"a{i}/first")
        out.first_failure = json.loads(first) if first else None
        if rank == 0:
            rcs = [co.get(f"a{i}/rc/{r}") for r in range(world)]
            out.rcs = [int(v) if v is not None else None for v in rcs]
            recs = [co.get(f"a{i}/failrec/{r}") for r in range(world)]
            out.failures = [json.loads(v) for v in recs if v]
    co.leave("end")
    return -1, outcomes


def annotate(line: dict, attempts: list, ok_index: int, outcomes: list) -> dict:
    """The successful attempt's JSON line + which path produced it and why earlier ones failed."""
    line = dict(line)
    line["dist_path"] = attempts[ok_index].name
    line["first_attempt_rc"] = 0
    if ok_index > 0:
        f0 = outcomes[0].first_failure or {}
        line["first_attempt_rc"] = f0.get("rc", outcomes[0].rc)
        line["failed_attempts"] = []
        for j in range(ok_index):
            f = outcomes[j].first_failure or {}
            fails = outcomes[j].failures or ([f] if f else [])
            line["failed_attempts"].append({
                "path": attempts[j].name, "failed_rank": f.get("rank"), "rc": f.get("rc", outcomes[j].rc),
                "rank_rcs": outcomes[j].rcs, "stderr_tail": f.get("stderr_tail", outcomes[j].stderr_tail[-12:]),
                "failed_ranks": [{"rank": x.get("rank"), "rc": x.get("rc"), "stderr_tail": x.get("stderr_tail", [])[-6:]}
                                 for x in fails]})
    return line
