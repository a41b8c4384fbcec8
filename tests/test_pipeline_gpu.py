"""The MLProbs pipeline driver on the GPU: every aligner call of the pipeline
(-G, -p 0|1 and each region's quickprobs) forced onto the device
(MLP_HOST_MAX_CELLS=0, one device context shared by the calls of a run),
against the reference pipeline's fixtures (tests/golden/pipeline, see
tests/test_pipeline.py): every stage and the final MSA bytes."""
import os

import pytest

from test_pipeline import ENV, check_trace, families, load, run_pipeline

pytestmark = pytest.mark.gpu

GPU_ENV = dict(ENV, MLP_HOST_MAX_CELLS='0', MLP_SCRATCH_GB='8')


@pytest.mark.parametrize('tag', families())
def test_pipeline_device_path(tag, tmp_path):
    rec = load(tag)
    res, tr = run_pipeline(tag, str(tmp_path), env=GPU_ENV)
    check_trace(rec, tr, tag)
    assert res == rec['final'], tag
