"""Argument validation shared by the accountant (reference
pipeline_dp/input_validators.py:17-34)."""


def validate_epsilon_delta(epsilon: float, delta: float, obj_name: str) -> None:
    if epsilon <= 0:
        raise ValueError(f"{obj_name}: epsilon must be positive, not {epsilon}.")
    if delta < 0:
        raise ValueError(f"{obj_name}: delta must be non-negative, not {delta}.")
    if delta >= 1:
        raise ValueError(f"{obj_name}: delta must be less than 1, not {delta}.")
