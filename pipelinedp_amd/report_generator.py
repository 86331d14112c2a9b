"""Explain-computation reports (reference pipeline_dp/report_generator.py).

Stages may be strings or zero-argument callables; callables are evaluated
when the report is rendered, i.e. after ``compute_budgets()`` when the
eps/delta they mention exist.
"""
from typing import Callable, Optional, Union

from .aggregate_params import parameters_to_readable_string


class ReportGenerator:

    def __init__(self, params, method_name: str, is_public_partition: Optional[bool] = None):
        self._params_str = parameters_to_readable_string(params, is_public_partition) if params else None
        self._method_name = method_name
        self._stages = []

    def add_stage(self, stage_description: Union[Callable, str]) -> None:
        self._stages.append(stage_description)

    def report(self) -> str:
        if not self._params_str:
            return ""
        out = [f"DPEngine method: {self._method_name}", self._params_str, "Computation graph:"]
        for i, stage in enumerate(self._stages, start=1):
            out.append(f" {i}. {stage() if callable(stage) else stage}")
        return "\n".join(out)


class ExplainComputationReport:
    """Output argument of DPEngine.aggregate(out_explain_computaton_report=)."""

    def __init__(self):
        self._report_generator = None

    def _set_report_generator(self, report_generator: ReportGenerator):
        self._report_generator = report_generator

    def text(self) -> str:
        if self._report_generator is None:
            raise ValueError("The report_generator is not set.\nWas this object"
                             " passed as an argument to DP aggregation method?")
        try:
            return self._report_generator.report()
        except Exception as e:
            raise ValueError("Explain computation report failed to be generated"
                             ".\nWas BudgetAccountant.compute_budget() called?") from e
