"""Physics presets of the four reference systems and the benchmark configs.

Values are the reference drivers' defaults (argparse in each */arguments.py plus the scaling done in
the drivers) — the runtime replacement of setupC.py's compile-time macros.
"""
from __future__ import annotations

from dataclasses import asdict, dataclass, replace
from math import pi

HO, IHO, QO, IQO = 0, 1, 2, 3
FAMILY_NAMES = {HO: "harmonic", IHO: "inverted_harmonic", QO: "quartic", IQO: "inverted_quartic"}


@dataclass(frozen=True)
class Physics:
    family: int
    n_max: int = 0              # Fock basis size - 1
    omega: float = pi           # Fock: args.omega * pi (IHO/main_parallel.py:30,42)
    x_max: float = 0.0          # grid
    grid_size: float = 0.0
    lambda_: float = 0.0        # grid: args.lambda * pi (IQO/main_parallel.py:29)
    mass: float = 0.0           # grid: args.mass / pi (IQO/main_parallel.py:31)
    moment_order: int = 5       # IQO/arguments.py: --input_moment_order
    gamma: float = pi           # args.gamma * pi
    time_steps: int = 1440      # dt = 1 / time_steps
    n_con: int = 18             # control steps per unit time
    f_max: float = 5.0          # convert_to_force spacing F_max / 10 (IHO/RL.py:107-111)
    n_actions: int = 21
    a_mode: int = 0             # 0 = reference MKL descriptor semantics, 1 = exact A
    precision: int = 0          # 0 = fp64 (the reference's), 1 = fp32 (config C5; Fock families)

    @property
    def dt(self) -> float:
        return 1.0 / self.time_steps

    @property
    def control_interval(self) -> int:
        # IHO/main_parallel.py:113-118, IQO/main_parallel.py:85-90
        assert self.time_steps % self.n_con == 0
        return round(self.time_steps / self.n_con)

    @property
    def fock(self) -> bool:
        return self.family in (HO, IHO)

    @property
    def dim(self) -> int:
        if self.fock:
            return self.n_max + 1
        return 2 * int(self.x_max / self.grid_size + 0.5) + 1

    @property
    def n_obs(self) -> int:
        if self.fock:
            return 5
        m = self.moment_order
        return (2 + m + 1) * m // 2

    @property
    def xth(self) -> float:
        """Termination threshold: IHO |<x>| > F_max (IHO/main_parallel.py:190);
        IQO outside-probability window (F_max/|lambda|/4*pi)^(1/3) (IQO/main_parallel.py:150)."""
        if self.family == IHO:
            return self.f_max
        if self.family == IQO:
            return (self.f_max / abs(self.lambda_) / 4 * pi) ** (1 / 3)
        return 0.0

    def force(self, action: int) -> float:
        half = self.n_actions // 2
        return (action - half) * (self.f_max / half)

    def with_(self, **kw) -> "Physics":
        return replace(self, **kw)

    def asdict(self):
        return asdict(self)


# driver defaults (HO/arguments.py, IHO/arguments.py, QO/arguments.py, IQO/arguments.py)
DEFAULTS = {
    HO: Physics(HO, n_max=70, gamma=1 * pi, time_steps=1440, f_max=5.0),
    IHO: Physics(IHO, n_max=180, gamma=2 * pi, time_steps=1440, f_max=8.0),
    QO: Physics(QO, x_max=8.5, grid_size=0.1, lambda_=0.04 * pi, mass=1 / pi, gamma=0.01 * pi,
                time_steps=1440, f_max=5.0),
    IQO: Physics(IQO, x_max=13.0, grid_size=0.05, lambda_=-0.01 * pi, mass=1 / pi, gamma=1 * pi,
                 time_steps=2880, f_max=5.0),
}

# BASELINE.json configs (SURVEY.md §8 sizes)
BENCH_CONFIGS = {
    "C1": dict(physics=DEFAULTS[HO].with_(n_max=255), batch=1),
    "C2": dict(physics=DEFAULTS[IHO].with_(n_max=511), batch=4096),
    # C3's fine grid (h = 8.5/512) is only stable for dt <= 1/11520: at the driver's 1/1440 every env Fails
    # within 1000 steps (oracle alike, tests/test_gpu_parity.py), so the workload runs at the stable dt
    # (control interval 640 physics steps)
    "C3": dict(physics=DEFAULTS[QO].with_(x_max=8.5, grid_size=8.5 / 512, time_steps=11520), batch=16384),
    "C4": dict(physics=DEFAULTS[IQO].with_(x_max=12.8, grid_size=0.05), batch=65536),
    "C5": dict(physics=DEFAULTS[IHO].with_(n_max=2047, precision=1), batch=262144),
    "metric": dict(physics=DEFAULTS[IHO].with_(n_max=511), batch=65536),
    # diagnostic (not a BASELINE config): C5's fp32 IHO kernel at N = 1024, R = 16 rows per lane, two waves per SIMD —
    # the per-wave side of C5's cost split (profiles/r06_C5r16_*)
    "C5r16": dict(physics=DEFAULTS[IHO].with_(n_max=1023, precision=1), batch=32768),
}
