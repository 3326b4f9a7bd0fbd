"""nifty_amd — MI355X-native geoVI/MGVI sampling hot path with the NIFTy 8.5
classic API (Field / LinearOperator / EndomorphicOperator / Energy,
SimpleCorrelatedField, draw_samples, SampledKLEnergy).

Import as ``import nifty_amd as ift`` (the package directory is
``joss-nifty_amd/``; ``nifty_amd.py`` at the repo root is the import shim).
Hot-path arithmetic runs in ``libnifty_amd.so`` (hand-written HIP kernels for
gfx950, C ABI in include/nifty_amd.h); PyTorch provides device memory,
streams and torch.distributed.
"""
from . import config, random
from .config import update as config_update
from .domain_tuple import DomainTuple
from .domains import DOFSpace, Domain, PowerSpace, RGSpace, StructuredDomain, UnstructuredDomain
from .ducc_dispatch import nthreads, set_nthreads
from .field import Field
from .library.correlated_fields import CorrelatedFieldMaker, _SlopeRemover, _SpecialSum, _TwoLogIntegrations
from .library.correlated_fields_simple import CFJacobian, SimpleCorrelatedField
from .library.los_response import LOSResponse
from .linearization import Linearization
from .logger import logger
from .minimization.conjugate_gradient import ConjugateGradient
from .minimization.descent_minimizers import DescentMinimizer, NewtonCG, SteepestDescent
from .minimization.energy import Energy
from .minimization.energy_adapter import EnergyAdapter
from .minimization.iteration_controllers import (AbsDeltaEnergyController, DeltaEnergyController,
                                                 EnergyHistory, GradientNormController,
                                                 GradInfNormController, IterationController)
from .minimization.kl_energies import SampledKLEnergy, SampledKLEnergyClass, draw_samples
from .minimization.line_search import LineSearch
from .minimization.quadratic_energy import QuadraticEnergy
from .minimization.optimize_kl import optimize_kl
from .minimization.sample_list import ResidualSampleList, SampleList
from .probing import StatCalculator, approximation2endo, probe_diagonal
from .multi_domain import MultiDomain
from .multi_field import MultiField
from .operators.adder import Adder
from .operators.block_diagonal_operator import BlockDiagonalOperator
from .operators.chain_operator import ChainOperator
from .operators.contraction_operator import ContractionOperator, IntegrationOperator
from .operators.diagonal_operator import DiagonalOperator
from .operators.distributors import DOFDistributor, PowerDistributor
from .operators.endomorphic_operator import EndomorphicOperator
from .operators.energy_operators import (EnergyOperator, GaussianEnergy, LikelihoodEnergyOperator,
                                         PoissonianEnergy, QuadraticFormOperator, Squared2NormOperator,
                                         StandardHamiltonian)
from .operators.harmonic_operators import (FFTOperator, HarmonicSmoothingOperator, HarmonicTransformOperator,
                                           HartleyOperator)
from .operators.linear_operator import LinearOperator
from .operators.normal_operators import LognormalTransform, NormalTransform
from .operators.operator import Operator
from .operators.operator_adapter import OperatorAdapter
from .operators.sampling_enabler import SamplingEnabler
from .operators.sandwich_operator import SandwichOperator
from .operators.scaling_operator import ScalingOperator
from .operators.simple_linear_operators import (ConjugationOperator, FieldAdapter, GeometryRemover,
                                                NullOperator, PartialExtractor, Realizer, VdotOperator,
                                                ducktape)
from .operators.sum_operator import SumOperator
from .operators.value_inserter import ValueInserter
from .sugar import (domain_union, exp, from_random, full, is_fieldlike, is_linearization, is_operator, log,
                    makeDomain, makeField, makeOp, sigmoid, sqrt, tanh)
from .utilities import TorchComm, allreduce_sum, myassert, shareRange

__version__ = "8.5+mi355x.r1"
