"""Utilities: synthetic clouds, timers (reference stopwatch.h), logging, dataset paths."""
from __future__ import annotations

import json
import logging
import os
import sys
import time
from pathlib import Path

import torch

REPO = Path(__file__).resolve().parents[2]
DATA = REPO / "data"


def dataset(name: str) -> Path:
    """Path of a shipped dataset (``pts20K.xyz`` is the reference's only shipped cloud)."""
    return DATA / name


def uniform_cloud(n: int, seed: int = 0, device="cpu", lo: float = 0.0, hi: float = 1000.0) -> torch.Tensor:
    """Uniform random points in [lo, hi)^3 (float32), generated on ``device``."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.rand((n, 3), generator=g, device=device, dtype=torch.float32) * (hi - lo) + lo


def blue_cloud(n: int, seed: int = 0, device="cpu") -> torch.Tensor:
    """Blue-noise stand-in: one jittered point per lattice cell (bounded minimum spacing),
    for the missing 300k/900k_blue_cube.xyz files of the reference (.MISSING_LARGE_BLOBS)."""
    m = max(1, int(round(n ** (1 / 3) + 0.4999)))
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    cells = torch.randperm(m ** 3, generator=g)[:n]
    ijk = torch.stack([cells % m, (cells // m) % m, cells // (m * m)], 1).float()
    jit = (torch.rand((n, 3), generator=g) - 0.5) * 0.7
    return ((ijk + 0.5 + jit) * (1000.0 / m)).to(device)


def clustered_cloud(n: int, seed: int = 0, device="cpu") -> torch.Tensor:
    """Gaussian clusters + 10% uniform background (stress case for the grid)."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    nc = max(1, n // 5000)
    centers = 100 + 800 * torch.rand((nc, 3), generator=g)
    sig = 5 + 40 * torch.rand((nc, 1), generator=g)
    which = torch.randint(0, nc, (n,), generator=g)
    pts = centers[which] + sig[which] * torch.randn((n, 3), generator=g)
    bg = torch.rand(n, generator=g) < 0.1
    pts[bg] = 1000 * torch.rand((int(bg.sum()), 3), generator=g)
    return pts.clamp(0, 1000).to(device)


def surface_cloud(n: int, seed: int = 0, device="cpu") -> torch.Tensor:
    """Points on 2-D surfaces in the [0,1000]^3 cube (a sphere and a tilted plane), the shape of
    scanned / meshed data: a uniform 3-D grid over the bbox puts tens of points in every
    occupied cell (the occupancy-adaptive grid refines it)."""
    g = torch.Generator(device="cpu")
    g.manual_seed(seed)
    ns = n * 2 // 3
    v = torch.randn((ns, 3), generator=g)
    sphere = 500 + 400 * v / v.norm(dim=1, keepdim=True)
    uv = torch.rand((n - ns, 2), generator=g) * 1000
    plane = torch.stack([uv[:, 0], uv[:, 1], 200 + 0.3 * uv[:, 0] + 0.1 * uv[:, 1]], 1)
    return torch.cat([sphere, plane]).clamp(0, 1000).to(device)


class Stopwatch:
    """RAII wall-clock timer (reference stopwatch.h:11-43, but monotonic and sub-ms):
    prints ``task...`` on entry and ``task: X ms`` on exit; ``tick()`` prints deltas."""

    def __init__(self, task: str, verbose: bool = True, file=sys.stderr):
        self.task, self.verbose, self.file = task, verbose, file
        self.t0 = self.last = 0.0
        self.elapsed_ms = 0.0

    def __enter__(self):
        if self.verbose:
            print(f"{self.task}...", file=self.file)
        self.t0 = self.last = time.perf_counter()
        return self

    def tick(self, label: str = "") -> float:
        now = time.perf_counter()
        d = (now - self.last) * 1e3
        self.last = now
        if self.verbose:
            print(f"{self.task} {label}: {d:.3f} ms", file=self.file)
        return d

    def __exit__(self, *exc):
        self.elapsed_ms = (time.perf_counter() - self.t0) * 1e3
        if self.verbose:
            print(f"{self.task}: {self.elapsed_ms:.3f} ms", file=self.file)
        return False


class DeviceTimer:
    """hipEvent-based timer on the current stream (device time, no host sync until read)."""

    def __init__(self):
        self.a = torch.cuda.Event(enable_timing=True)
        self.b = torch.cuda.Event(enable_timing=True)

    def __enter__(self):
        self.a.record()
        return self

    def __exit__(self, *exc):
        self.b.record()
        return False

    @property
    def ms(self) -> float:
        self.b.synchronize()
        return self.a.elapsed_time(self.b)


def get_logger(name: str = "knearests") -> logging.Logger:
    """Leveled logger of the package (``knearests`` or a ``knearests.*`` child). The level comes
    from env ``KN_LOG`` (DEBUG / INFO / WARNING / ERROR, default WARNING); the same variable sets
    the native library's verbosity (``kn_default_config``: DEBUG -> 2, INFO -> 1)."""
    root = logging.getLogger("knearests")
    if not root.handlers:
        h = logging.StreamHandler(sys.stderr)
        h.setFormatter(logging.Formatter("[%(name)s %(levelname)s] %(message)s"))
        root.addHandler(h)
        lvl = os.environ.get("KN_LOG", "WARNING").upper()
        root.setLevel(lvl if lvl in ("DEBUG", "INFO", "WARNING", "ERROR", "CRITICAL") else "WARNING")
        root.propagate = False  # one line per record even when the application configures logging
    return logging.getLogger(name)


def emit_json(obj: dict, file=sys.stdout) -> None:
    print(json.dumps(obj), file=file, flush=True)


__all__ = ["dataset", "uniform_cloud", "blue_cloud", "clustered_cloud", "Stopwatch", "DeviceTimer",
           "get_logger", "emit_json", "REPO", "DATA"]
