"""pipelinedp_amd — MI355X-native DPEngine.aggregate hot path of PipelineDP.

Host API mirrors ``pipeline_dp`` (reference pipeline_dp/__init__.py:14-34);
compute runs in libpdp_hip.so (hand-written HIP for gfx950) behind the
HipBackend plugin.
"""
from pipelinedp_amd.aggregate_params import (AggregateParams, CountParams, MeanParams, MechanismType, Metric,
                                             Metrics, NoiseKind, NormKind, PartitionSelectionStrategy,
                                             PrivacyIdCountParams, SelectPartitionsParams, SumParams,
                                             VarianceParams)
from pipelinedp_amd.budget_accounting import BudgetAccountant, MechanismSpec, NaiveBudgetAccountant
from pipelinedp_amd.columnar import ColumnarData
from pipelinedp_amd.dp_engine import DataExtractors, DPEngine, DPResult
from pipelinedp_amd.pipeline_backend import Annotator, HipBackend, PipelineBackend, register_annotator
from pipelinedp_amd.private_collection import PrivateCollection, make_private
from pipelinedp_amd.report_generator import ExplainComputationReport

__version__ = "0.1.0"
