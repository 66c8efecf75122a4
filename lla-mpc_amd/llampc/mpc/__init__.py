from llampc.mpc.evaluate_models_vectorized import evaluate_models_vectorized  # noqa: F401
from llampc.mpc.bank import ModelBank, generate_bank, shard_range  # noqa: F401
from llampc.mpc.plan import PlanResult, plan  # noqa: F401
from llampc.mpc.planner import ConstantSpeed  # noqa: F401
from llampc.mpc.controller import (LLAMPC, CandidateGenerator, DeviceController,  # noqa: F401
                                   ExponentialSmoother, MuEstimator, update_friction, FRICTION_CASES)
from llampc.mpc.nmpc import setupNLP  # noqa: F401
