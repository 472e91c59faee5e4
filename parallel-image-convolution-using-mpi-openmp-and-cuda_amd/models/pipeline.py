"""Multi-stage convolution pipelines.

The reference applies ONE filter `reps` times (the gaussian is active, the box
and "edge" filters are commented-out alternatives: ``mpi/mpi_convolution.c:
88-102``).  A ``FilterPipeline`` chains stages — e.g. ``"gaussian:10,edge:1"``
smooths ten times, then runs one edge pass — each stage executed by the same
engines (fused SWAR kernel for gaussian stages, exact generic kernels for the
others), so a pipeline is exactly the composition of single-filter runs.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Iterable, List, Optional, Sequence, Tuple, Union

from .filters import Filter, get_filter

StageSpec = Union[str, Tuple[Union[str, Filter, Tuple[Sequence[int], int]], int]]


@dataclass(frozen=True)
class Stage:
    filter: Filter
    reps: int


class FilterPipeline:
    def __init__(self, stages: Iterable[StageSpec]):
        parsed: List[Stage] = []
        for st in stages:
            if isinstance(st, str):
                name, _, reps = st.partition(":")
                parsed.append(Stage(get_filter(name.strip()), int(reps) if reps else 1))
            else:
                flt, reps = st
                parsed.append(Stage(get_filter(flt), int(reps)))
        for s in parsed:
            if s.reps < 0:
                raise ValueError("stage repetitions must be >= 0")
        self.stages: Tuple[Stage, ...] = tuple(parsed)

    @classmethod
    def from_spec(cls, spec: str) -> "FilterPipeline":
        """``"gaussian:10,edge:1"`` (a stage without ``:n`` runs once)."""
        return cls([p for p in spec.split(",") if p.strip()])

    @property
    def total_reps(self) -> int:
        return sum(s.reps for s in self.stages)

    def __repr__(self) -> str:
        return "FilterPipeline(" + ",".join(f"{s.filter.name}:{s.reps}" for s in self.stages) + ")"

    def apply(self, image, backend: str = "auto", device: Optional[int] = None):
        """Run every stage in order; returns the same container type as ``image``."""
        from ..ops.stencil import convolve

        out = image
        for s in self.stages:
            if s.reps:
                out = convolve(out, s.reps, s.filter, backend=backend, device=device)
        return out

    def reference(self, image):
        """Independent NumPy oracle of the whole pipeline."""
        from ..ops.reference import numpy_convolve

        out = image
        for s in self.stages:
            out = numpy_convolve(out, s.reps, s.filter)
        return out
