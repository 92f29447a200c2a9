"""End-to-end block validation with the GPU backends (HBM UTXO index + batched P-256 kernels)."""
import asyncio
import argparse

import pytest


@pytest.mark.gpu
def test_verify_bench_pipeline_on_gpu(gpu, monkeypatch):
    from decimal import Decimal
    from upow_amd import constants
    from upow_amd.ledger import manager
    monkeypatch.setattr(constants, 'START_DIFFICULTY', Decimal('4.0'))
    monkeypatch.setattr(manager, 'START_DIFFICULTY', Decimal('4.0'))
    from upow_amd.bench_verify import run_verify_bench
    from upow_amd.parallel.dist import DistContext
    args = argparse.Namespace(steps=1, warmup=1, txs=600)
    out = run_verify_bench(args, DistContext())
    assert out['config']['utxo_backend'] == 'gpu' and out['config']['device'] == 'gpu'
    assert out['value'] > 0
