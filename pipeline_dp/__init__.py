"""``import pipeline_dp`` for callers of the reference (PipelineDP 0.2.1rc3).

The reference's public names (pipeline_dp/__init__.py:14-34) resolved to the
MI355X implementation in ``pipelinedp_amd``: existing ``DPEngine.aggregate``,
``AggregateParams`` + ``DataExtractors`` and ``make_private(...).sum/count/
mean/variance/privacy_id_count`` code runs unchanged except for the backend
object, ``pipeline_dp.HipBackend()`` in place of ``pipeline_dp.LocalBackend()``
(INTEGRATION.md §3).  The reference's submodules that callers import by name
(``pipeline_dp.aggregate_params``, ``budget_accounting``, ``dp_engine``,
``pipeline_backend``, ``report_generator``) map to the same modules here.
"""
import sys as _sys

import pipelinedp_amd as _impl
from pipelinedp_amd import *  # noqa: F401,F403
from pipelinedp_amd import (AggregateParams, Annotator, BudgetAccountant, ColumnarData, CountParams,  # noqa: F401
                            DataExtractors, DPEngine, ExplainComputationReport, HipBackend, MeanParams,
                            MechanismSpec, MechanismType, Metric, Metrics, NaiveBudgetAccountant, NoiseKind,
                            NormKind, PartitionSelectionStrategy, PipelineBackend, PrivacyIdCountParams,
                            SelectPartitionsParams, SumParams, VarianceParams, make_private,
                            register_annotator)
from pipelinedp_amd import aggregate_params, budget_accounting, dp_engine, pipeline_backend  # noqa: F401
from pipelinedp_amd import report_generator  # noqa: F401

for _name in ("aggregate_params", "budget_accounting", "dp_engine", "pipeline_backend", "report_generator"):
    _sys.modules[f"{__name__}.{_name}"] = getattr(_impl, _name)

__version__ = _impl.__version__


def __getattr__(name):
    if name == "LocalBackend":
        raise AttributeError("pipeline_dp.LocalBackend is the reference's pure-Python backend; this package runs "
                             "DPEngine on the MI355X: use pipeline_dp.HipBackend()")
    raise AttributeError(name)
