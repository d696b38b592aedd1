"""H2OAssembly: a named pipeline of frame munging steps (reference h2o-py
h2o/assembly.py over water/rapids/Assembly.java).  ``fit`` runs the steps in
order on the device frame; the reference additionally ships the step list to
the server to emit a munging POJO, which needs the Java toolchain this
framework does not carry."""
from __future__ import annotations


class H2OAssembly:
    def __init__(self, steps):
        if not steps or not all(isinstance(s, (list, tuple)) and len(s) == 2 for s in steps):
            raise ValueError("steps must be a non-empty list of (name, transformer) pairs")
        self.steps = list(steps)
        self.id = None
        self.fuzzy = None

    @property
    def names(self):
        return [name for name, _ in self.steps]

    def fit(self, fr):
        out = fr
        for _, step in self.steps:
            out = step.fit_transform(out)
        self.id = f"assembly_{id(self):x}"
        return out

    def to_pojo(self, pojo_name="", path="", get_jar=True):
        raise NotImplementedError("munging POJO export (Assembly.java) is not provided: the fitted steps run on "
                                  "the GPU frame directly; score models through their MOJO")
