"""Apache Arrow IPC logger for EvoXVis (reference ``monitors/evoxvis_monitor.py:11-224``).

Writes one row per generation: ``generation`` (uint64), ``fitness`` and optionally
``population`` as fixed-size binary blobs (dtype recorded in the schema
metadata), ``duration`` (seconds since the first record) and scalar metrics.
Rows are buffered and written in record batches of ``batch_size`` with optional
lz4/zstd compression.  Unlike the reference (which defines no ``hooks()`` and so
cannot be registered) this is a proper :class:`Monitor`
hooked on ``post_ask``/``post_eval``.
"""
from __future__ import annotations

import tempfile
import time
from pathlib import Path
from typing import Optional

import numpy as np
import pyarrow as pa
import torch

from ..core import Monitor


class EvoXVisMonitor(Monitor):
    def __init__(self, base_filename: str, out_dir: Optional[str] = None, out_type: str = "file", batch_size: int = 64, compression: Optional[str] = None, record_population: bool = True, record_time: bool = True):
        super().__init__()
        self.batch_size = batch_size
        self.record_population = record_population
        self.record_time_flag = record_time
        base = Path(tempfile.gettempdir()).joinpath("evox") if out_dir is None else Path(out_dir)
        base.mkdir(parents=True, exist_ok=True)
        i = 0
        while base.joinpath(f"{base_filename}_{i}.arrow").exists():
            i += 1
        self.path = str(base.joinpath(f"{base_filename}_{i}.arrow"))
        self.sink = pa.OSFile(self.path, "wb")
        self.out_type = out_type
        self.comp_alg = compression
        self.schema = None
        self.writer = None
        self.is_closed = False
        self.generation_counter = 0
        self.rows = []
        self._pending_pop = None
        self.ref_time = None
        self.opt_direction = 1

    def hooks(self):
        return ["post_ask", "post_eval"]

    def set_opt_direction(self, opt_direction):
        self.opt_direction = opt_direction

    def post_ask(self, _state, cand_sol):
        if self.record_population:
            self._pending_pop = cand_sol

    def post_eval(self, _state, _cand_sol, _transformed, fitness):
        self.record(fitness, self._pending_pop)

    def record_time(self):
        now = time.perf_counter()
        if self.ref_time is None:
            self.ref_time = now
        return now - self.ref_time

    def record(self, fitness, population=None, metrics: dict = None):
        fit = fitness.detach().to("cpu").numpy()
        row = {"generation": self.generation_counter, "fitness": fit.tobytes(), "fitness_dtype": str(fit.dtype), "fitness_shape": fit.shape}
        if population is not None:
            pop = population.detach().to("cpu").numpy()
            row.update(population=pop.tobytes(), population_dtype=str(pop.dtype), population_shape=pop.shape)
        if self.record_time_flag:
            row["duration"] = self.record_time()
        if metrics:
            row["metrics"] = {k: float(v) for k, v in metrics.items()}
        self.rows.append(row)
        self.generation_counter += 1
        if len(self.rows) >= self.batch_size:
            self._write_batch()

    def _init_writer(self, r0):
        fields = [("generation", pa.uint64()), ("fitness", pa.binary(len(r0["fitness"])))]
        meta = {"population_size": str(r0["fitness_shape"][0]), "fitness_dtype": r0["fitness_dtype"], "fitness_shape": ",".join(map(str, r0["fitness_shape"]))}
        if "population" in r0:
            fields.append(("population", pa.binary(len(r0["population"]))))
            meta["population_dtype"] = r0["population_dtype"]
            meta["population_shape"] = ",".join(map(str, r0["population_shape"]))
        if "duration" in r0:
            fields.append(("duration", pa.float64()))
            meta["begin_time"] = str(time.time())
        self.metric_names = sorted(r0.get("metrics", {}).keys())
        for n in self.metric_names:
            fields.append((n, pa.float64()))
        if self.metric_names:
            meta["metrics"] = "_".join(self.metric_names)
        self.schema = pa.schema(fields, metadata=meta)
        opts = pa.ipc.IpcWriteOptions(compression=self.comp_alg)
        if self.out_type == "file":
            self.writer = pa.ipc.new_file(self.sink, self.schema, options=opts)
        else:
            self.writer = pa.ipc.new_stream(self.sink, self.schema, options=opts)

    def _write_batch(self):
        if not self.rows:
            return
        if self.schema is None:
            self._init_writer(self.rows[0])
        cols = [[r["generation"] for r in self.rows], [r["fitness"] for r in self.rows]]
        if "population" in self.rows[0]:
            cols.append([r["population"] for r in self.rows])
        if "duration" in self.rows[0]:
            cols.append([r["duration"] for r in self.rows])
        for n in self.metric_names:
            cols.append([r["metrics"][n] for r in self.rows])
        self.writer.write_batch(pa.record_batch(cols, schema=self.schema))
        self.rows = []

    def flush(self):
        self._write_batch()

    def close(self):
        if self.is_closed:
            return
        self._write_batch()
        if self.writer is not None:
            self.writer.close()
        self.sink.close()
        self.is_closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def read_evoxvis(path: str):
    """Load an EvoXVis arrow file back into numpy arrays (for tests / analysis)."""
    with pa.OSFile(path, "rb") as f:
        table = pa.ipc.open_file(f).read_all()
    meta = {k.decode(): v.decode() for k, v in (table.schema.metadata or {}).items()}
    fshape = tuple(int(x) for x in meta["fitness_shape"].split(","))
    fit = [np.frombuffer(b.as_py(), dtype=meta["fitness_dtype"]).reshape(fshape) for b in table.column("fitness")]
    out = {"generation": table.column("generation").to_pylist(), "fitness": fit, "meta": meta}
    if "population" in table.column_names:
        pshape = tuple(int(x) for x in meta["population_shape"].split(","))
        out["population"] = [np.frombuffer(b.as_py(), dtype=meta["population_dtype"]).reshape(pshape) for b in table.column("population")]
    if "duration" in table.column_names:
        out["duration"] = table.column("duration").to_pylist()
    return out
