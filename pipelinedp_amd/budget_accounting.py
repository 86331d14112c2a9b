"""Privacy budget accounting — stays on the host (north star).

Same semantics as the reference ``pipeline_dp/budget_accounting.py``:
lazy ``MechanismSpec`` objects (:35-99) whose eps/delta become readable only
after ``compute_budgets()``; nested weight scopes (:159-175, 261-286); naive
composition splitting eps by weight over all mechanisms and delta only over
mechanisms that use it (:368-396).
"""
import abc
import collections
import dataclasses
import logging
from typing import List, Optional

from . import aggregate_params as agg
from .input_validators import validate_epsilon_delta

Budget = collections.namedtuple("Budget", ["epsilon", "delta"])


@dataclasses.dataclass
class MechanismSpec:
    mechanism_type: agg.MechanismType
    _noise_standard_deviation: float = None
    _eps: float = None
    _delta: float = None
    _count: int = 1

    @property
    def noise_standard_deviation(self):
        if self._noise_standard_deviation is None:
            raise AssertionError("Noise standard deviation is not calculated yet.")
        return self._noise_standard_deviation

    @property
    def eps(self):
        if self._eps is None:
            raise AssertionError("Privacy budget is not calculated yet.")
        return self._eps

    @property
    def delta(self):
        if self._delta is None:
            raise AssertionError("Privacy budget is not calculated yet.")
        return self._delta

    @property
    def count(self):
        return self._count

    @property
    def is_computed(self) -> bool:
        return self._eps is not None

    def set_eps_delta(self, eps: float, delta: Optional[float]) -> None:
        if eps is None:
            raise AssertionError("eps must not be None.")
        self._eps = eps
        self._delta = delta

    def use_delta(self) -> bool:
        return self.mechanism_type != agg.MechanismType.LAPLACE


@dataclasses.dataclass
class MechanismSpecInternal:
    sensitivity: float
    weight: float
    mechanism_spec: MechanismSpec


class BudgetAccountantScope:
    """``with accountant.scope(weight):`` — mechanisms requested inside share
    ``weight`` of the parent's budget, proportionally to their own weights."""

    def __init__(self, accountant, weight):
        self.weight = weight
        self.accountant = accountant
        self.mechanisms: List[MechanismSpecInternal] = []

    def __enter__(self):
        self.accountant._enter_scope(self)
        return self

    def __exit__(self, exc_type, exc_val, exc_tb):
        self.accountant._exit_scope()
        if self.mechanisms:
            factor = self.weight / sum(m.weight for m in self.mechanisms)
            for m in self.mechanisms:
                m.weight *= factor


class BudgetAccountant(abc.ABC):

    def __init__(self, total_epsilon: float, total_delta: float, num_aggregations: Optional[int],
                 aggregation_weights: Optional[list]):
        validate_epsilon_delta(total_epsilon, total_delta, "BudgetAccountant")
        self._total_epsilon = total_epsilon
        self._total_delta = total_delta
        self._scopes_stack = []
        self._mechanisms = []
        self._finalized = False
        if num_aggregations is not None and aggregation_weights is not None:
            raise ValueError("'num_aggregations' and 'aggregation_weights' can not be set "
                             "simultaneously.\nIf you wish all aggregations in the pipeline "
                             "to have equal budgets, specify the total number of aggregations"
                             "with 'n_aggregations'.\nIf you wish to have different budgets "
                             "for different aggregations, specify them with 'aggregation_weights'")
        if num_aggregations is not None and num_aggregations <= 0:
            raise ValueError(f"'num_aggregations'={num_aggregations}, but it has to be positive.")
        self._expected_num_aggregations = num_aggregations
        self._expected_aggregation_weights = aggregation_weights
        self._actual_aggregation_weights = []

    @abc.abstractmethod
    def request_budget(self, mechanism_type: agg.MechanismType, sensitivity: float = 1, weight: float = 1,
                       count: int = 1, noise_standard_deviation: Optional[float] = None) -> MechanismSpec:
        pass

    @abc.abstractmethod
    def compute_budgets(self):
        pass

    def scope(self, weight: float) -> BudgetAccountantScope:
        return BudgetAccountantScope(self, weight)

    def _compute_budget_for_aggregation(self, weight: float) -> Optional[Budget]:
        self._actual_aggregation_weights.append(weight)
        if self._expected_num_aggregations:
            k = self._expected_num_aggregations
            return Budget(self._total_epsilon / k, self._total_delta / k)
        if self._expected_aggregation_weights:
            ratio = weight / sum(self._expected_aggregation_weights)
            return Budget(self._total_epsilon * ratio, self._total_delta * ratio)
        return None

    def _check_aggregation_restrictions(self):
        actual = self._actual_aggregation_weights
        if self._expected_num_aggregations:
            if len(actual) != self._expected_num_aggregations:
                raise ValueError(f"'num_aggregations'({self._expected_num_aggregations}) in "
                                 f"the constructor of BudgetAccountant is different from the"
                                 f" actual number of aggregations in the pipeline"
                                 f"({len(actual)}). If 'n_aggregations' is "
                                 f"specified, you must have that many aggregations in the "
                                 f"pipeline.")
            if not all(w == 1 for w in actual):
                raise ValueError(f"Aggregation weights = {actual}. If 'num_aggregations' is"
                                 f" set in the constructor of BudgetAccountant, all "
                                 f"aggregation weights have to be 1. If you'd like to have "
                                 f"different weights use 'aggregation_weights'.")
        expected = self._expected_aggregation_weights
        if expected:
            if len(actual) != len(expected):
                raise ValueError(f"Length of 'aggregation_weights' in the constructor of "
                                 f"BudgetAccountant is {len(expected)} != "
                                 f"{len(actual)} the actual number of aggregations.")
            if not all(a == e for a, e in zip(actual, expected)):
                raise ValueError(f"'aggregation_weights' in the constructor of is "
                                 f"({expected}) is different from actual aggregation"
                                 f" weights ({actual}).If 'aggregation_weights' is "
                                 f"specified, they must be the same.")

    def _register_mechanism(self, mechanism: MechanismSpecInternal) -> MechanismSpecInternal:
        self._mechanisms.append(mechanism)
        for scope in self._scopes_stack:
            scope.mechanisms.append(mechanism)
        return mechanism

    def _enter_scope(self, scope):
        self._scopes_stack.append(scope)

    def _exit_scope(self):
        self._scopes_stack.pop()

    def _finalize(self):
        if self._finalized:
            raise Exception("compute_budgets can not be called twice.")
        self._finalized = True


class NaiveBudgetAccountant(BudgetAccountant):
    """Naive composition accountant (reference :289-396)."""

    def __init__(self, total_epsilon: float, total_delta: float, num_aggregations: Optional[int] = None,
                 aggregation_weights: Optional[list] = None):
        super().__init__(total_epsilon, total_delta, num_aggregations, aggregation_weights)

    def request_budget(self, mechanism_type: agg.MechanismType, sensitivity: float = 1, weight: float = 1,
                       count: int = 1, noise_standard_deviation: Optional[float] = None) -> MechanismSpec:
        if self._finalized:
            raise Exception("request_budget() is called after compute_budgets(). "
                            "Please ensure that compute_budgets() is called after DP "
                            "aggregations.")
        if noise_standard_deviation is not None:
            raise NotImplementedError("Count and noise standard deviation have not been implemented yet.")
        if mechanism_type == agg.MechanismType.GAUSSIAN and self._total_delta == 0:
            raise ValueError("The Gaussian mechanism requires that the pipeline delta is greater than 0")
        spec = MechanismSpec(mechanism_type=mechanism_type, _count=count)
        self._register_mechanism(MechanismSpecInternal(sensitivity=sensitivity, weight=weight, mechanism_spec=spec))
        return spec

    def compute_budgets(self):
        self._check_aggregation_restrictions()
        self._finalize()
        if not self._mechanisms:
            logging.warning("No budgets were requested.")
            return
        if self._scopes_stack:
            raise Exception("Cannot call compute_budgets from within a budget scope.")
        w_eps = sum(m.weight * m.mechanism_spec.count for m in self._mechanisms)
        w_delta = sum(m.weight * m.mechanism_spec.count for m in self._mechanisms if m.mechanism_spec.use_delta())
        for m in self._mechanisms:
            eps = self._total_epsilon * m.weight / w_eps if w_eps else 0
            delta = 0
            if m.mechanism_spec.use_delta() and w_delta:
                delta = self._total_delta * m.weight / w_delta
            m.mechanism_spec.set_eps_delta(eps, delta)


class PLDBudgetAccountant(BudgetAccountant):
    """Out of scope: experimental in the reference (:399-600), needs the
    absent dp_accounting package and is not DPEngine-compatible (:406)."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError("PLDBudgetAccountant is not part of the MI355X aggregate path; "
                                  "use NaiveBudgetAccountant.")
