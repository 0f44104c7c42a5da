import json

import pytest
import torch

import heat_amd as ht
from heat_amd import profiling


def test_counters_and_region(tmp_path):
    profiling.reset()
    profiling.enable()
    try:
        x = ht.arange(100, split=0, dtype=ht.float32)
        with profiling.region("sum"):
            s = ht.sum(x)
        assert float(s.item()) == pytest.approx(4950.0)
        c = profiling.counters()
        assert c["region:sum"]["calls"] == 1
        assert any(k in c for k in ("Allreduce", "allreduce")) or ht.MPI_WORLD.size == 1
        profiling.dump(str(tmp_path / "c.json"))
        assert "region:sum" in json.load(open(tmp_path / "c.json"))
    finally:
        profiling.disable()
    assert not profiling.enabled()


def test_fault_injection(monkeypatch):
    monkeypatch.setattr(profiling, "_fault", (ht.MPI_WORLD.rank, "Allreduce", 1))
    profiling._fault_calls.clear()
    profiling.enable()
    try:
        with pytest.raises(RuntimeError, match="HEAT_FAULT_INJECT"):
            ht.MPI_WORLD.Allreduce(ht.MPI.IN_PLACE, torch.ones(3), ht.MPI.SUM)
    finally:
        profiling.disable()
        profiling._fault_calls.clear()
