"""optimize_kl: the standard geoVI / MGVI driver with checkpoint and resume
(src/minimization/optimize_kl.py:51-412 and its helpers :415-758).

Per global iteration: draw n_samples (mirrored) samples around the current
mean -- the native batched CG / geoVI refinement of this package -- build
SampledKLEnergy, minimise it with kl_minimizer, keep the new mean and the
samples; MAP iterations (n_samples == 0) minimise the Hamiltonian with an
EnergyAdapter.  Every argument that the reference allows to be a function of
the iteration index still is.  With an output directory, each finished
iteration writes the sample list, the random state and the energy history
(checkpoint.py: the reference's layout and file stems, data-only files) and
`last_finished_iteration`; resume=True continues from there with the
identical random stream.

Not carried over (reporting only, SURVEY.md §2 OUT): matplotlib plots of the
energy / minisanity histories, the CountingOperator report and minisanity;
export_operator_outputs writes mean / std (and the samples) of each
operator as .npz instead of HDF5 / FITS."""
from inspect import signature
from os import makedirs
from os.path import isfile, join

import numpy as np

from ..domain_tuple import DomainTuple
from ..logger import logger
from ..multi_domain import MultiDomain
from ..multi_field import MultiField
from ..operators.energy_operators import StandardHamiltonian
from ..operators.operator import Operator
from ..sugar import from_random, full, makeDomain
from ..utilities import (check_MPI_equality, check_MPI_synced_random_state, get_MPI_params_from_comm,
                         myassert)
from . import checkpoint
from .descent_minimizers import DescentMinimizer
from .energy_adapter import EnergyAdapter
from .iteration_controllers import EnergyHistory, IterationController
from .kl_energies import SampledKLEnergy
from .minimizer import Minimizer
from .sample_list import ResidualSampleList, SampleList, _barrier


def optimize_kl(likelihood_energy, total_iterations, n_samples, kl_minimizer, sampling_iteration_controller,
                nonlinear_sampling_minimizer, constants=[], point_estimates=[], transitions=None,
                export_operator_outputs={}, output_directory=None, initial_position=None, initial_index=0,
                comm=None, inspect_callback=None, terminate_callback=None, plot_energy_history=True,
                plot_minisanity_history=True, save_strategy="last", return_final_position=False, resume=False,
                sanity_checks=True, dry_run=False):
    """optimize_kl.py:51-412 (same arguments and return values)."""
    if not isinstance(export_operator_outputs, dict):
        raise TypeError
    if "pickle" in export_operator_outputs:
        raise ValueError("The key `pickle` in `export_operator_outputs` is reserved.")
    if not isinstance(initial_index, int):
        raise TypeError
    if save_strategy not in ("all", "last"):
        raise ValueError(f"Save strategy '{save_strategy}' not supported.")
    if output_directory is None and resume:
        raise ValueError("Can only resume minimization if output_directory is not None")

    likelihood_energy = _make_callable(likelihood_energy)
    kl_minimizer = _make_callable(kl_minimizer)
    sampling_iteration_controller = _make_callable(sampling_iteration_controller)
    nonlinear_sampling_minimizer = _make_callable(nonlinear_sampling_minimizer)
    constants = _make_callable(constants)
    point_estimates = _make_callable(point_estimates)
    transitions = _make_callable(transitions)
    n_samples = _make_callable(n_samples)
    comm = _make_callable(comm)
    inspect_callback = _make_callable(inspect_callback)
    if terminate_callback is None:
        terminate_callback = _make_callable(False)

    mean = full(makeDomain({}), 0.) if initial_position is None else initial_position
    sl = _single_value_sample_list(mean, comm(initial_index))
    energy_history = EnergyHistory()

    if initial_index >= total_iterations:
        raise ValueError(f"Initial index is bigger than total iterations: {initial_index} >= {total_iterations}")
    if _nargs(transitions) != 1:
        raise ValueError(f"Transition takes 1 argument but {_nargs(transitions)} were given.")
    if _nargs(inspect_callback) not in (1, 2):
        raise ValueError(f"Inspect callback takes either 1 or 2 arguments but {_nargs(inspect_callback)}"
                         "were given.")
    if _nargs(terminate_callback) != 1:
        raise ValueError(f"Terminate callback takes 1 argument but {_nargs(terminate_callback)} were given.")
    if likelihood_energy(initial_index).target is not DomainTuple.scalar_domain():
        raise TypeError

    if sanity_checks:
        for it in range(initial_index, total_iterations):
            for obj, cls in ((likelihood_energy, Operator), (kl_minimizer, DescentMinimizer),
                             (nonlinear_sampling_minimizer, (DescentMinimizer, type(None))),
                             (constants, (list, tuple)), (point_estimates, (list, tuple)), (n_samples, int)):
                if not isinstance(obj(it), cls):
                    raise TypeError(f"{obj(it)} is not instance of {cls} but rather {type(obj(it))}")
            if sampling_iteration_controller(it) is None:
                myassert(n_samples(it) == 0)
            else:
                myassert(isinstance(sampling_iteration_controller(it), IterationController))
            myassert(likelihood_energy(it).target is DomainTuple.scalar_domain())

    out = output_directory
    stem = (lambda i: f"iteration_{i}") if save_strategy == "all" else (lambda i: "last")
    if out is not None:
        if _master(comm(initial_index)):
            for sub in ["pickle"] + list(export_operator_outputs.keys()):
                makedirs(join(out, sub), exist_ok=True)
        _barrier(comm(initial_index))
        lfile = join(out, "last_finished_iteration")
        if resume and isfile(lfile):
            with open(lfile) as f:
                last = int(f.read())
            initial_index = last + 1
            base = join(out, "pickle", stem(last))
            dom = likelihood_energy(min(last, total_iterations - 1)).domain
            if isfile(base + ".mean.npz"):
                mean = ResidualSampleList.load_mean(base, dom)
                sl = ResidualSampleList.load(base, comm(last), dom)
            else:
                sl = SampleList.load(base, comm(last), dom)
                mean = sl.local_item(0) if sl.n_local_samples else None
                mean = _bcast(mean, comm(last))
            checkpoint.set_random_state(checkpoint.load_json(join(out, "pickle", f"nifty_random_state_{stem(last)}.json")))
            energy_history = _history_from(checkpoint.load_json(join(out, "pickle", f"energy_history_{stem(last)}.json")))
            if initial_index == total_iterations:
                return (sl, mean) if return_final_position else sl

    for it in range(initial_index, total_iterations):
        lh = likelihood_energy(it)
        if not isinstance(lh.domain, MultiDomain):
            raise TypeError(f"Domain of likelihood_energy needs to be a MultiDomain, got\n{lh.domain}")
        t = transitions(it)
        mean = mean if t is None else t(sl)
        mean = _normal_initialize(mean, lh.domain)
        ham = StandardHamiltonian(lh, sampling_iteration_controller(it))
        minimizer = kl_minimizer(it)
        mean_iter = mean.extract(ham.domain)
        if dry_run:
            logger.info(f"Iteration {it} checked")
            continue
        cm = comm(it)
        # every rank runs the same iteration (optimize_kl.py:342-345); the
        # mean by a device checksum of each key, one allgather of tokens
        check_MPI_synced_random_state(cm)
        check_MPI_equality(lh.domain, cm)
        check_MPI_equality(mean.domain, cm)
        check_MPI_equality(mean, cm, hash_=True)
        sl = None
        if n_samples(it) == 0:
            e = EnergyAdapter(mean_iter, ham, constants=constants(it), want_metric=True)
            if cm is None:
                e, _ = minimizer(e)
                mean = MultiField.union([mean, e.position])
                sl = SampleList([mean])
                energy_history.append((it, e.value))
            else:
                # optimize_kl.py:343-355: rank 0 minimises, the others receive
                if _master(cm):
                    e, _ = minimizer(e)
                    energy_history.append((it, e.value))
                    mean = MultiField.union([mean, e.position])
                else:
                    mean = None
                _barrier(cm)
                mean = _bcast(mean, cm)
                sl = _single_value_sample_list(mean, cm)
        else:
            e = SampledKLEnergy(mean_iter, ham, n_samples(it), nonlinear_sampling_minimizer(it), comm=cm,
                                constants=constants(it), point_estimates=point_estimates(it))
            e, _ = minimizer(e)
            mean = MultiField.union([mean, e.position])
            sl = e.samples.at(mean)
            energy_history.append((it, e.value))

        if out is not None:
            _export_operators(out, stem(it), export_operator_outputs, sl)
            # a stem's previous files go first: with save_strategy "last" the
            # reference leaves a stale <stem>.mean (and surplus sample files)
            # behind when a sampled iteration is followed by a MAP one or by
            # fewer samples, and resume then reads them
            if _master(cm):
                _clear_stem(join(out, "pickle", stem(it)))
            _barrier(cm)
            sl.save(join(out, "pickle", stem(it)), overwrite=True)
            if _master(cm):
                checkpoint.save_json(join(out, "pickle", f"nifty_random_state_{stem(it)}.json"),
                                     checkpoint.random_state())
                checkpoint.save_json(join(out, "pickle", f"energy_history_{stem(it)}.json"),
                                     {"time_stamps": energy_history.time_stamps,
                                      "energy_values": energy_history.energy_values})
                with open(join(out, "last_finished_iteration"), "w") as f:
                    f.write(str(it))
        _barrier(cm)
        if _nargs(inspect_callback) == 1:
            inspect_callback(sl)
        else:
            inspect_callback(sl, it)
        _barrier(cm)
        if terminate_callback(it):
            break
        _barrier(cm)
    return (sl, mean) if return_final_position else sl


# ---------------------------------------------------------------- helpers
def _make_callable(obj):
    """optimize_kl.py:698-703"""
    if callable(obj) and not isinstance(obj, (Minimizer, IterationController, Operator)):
        return obj
    return lambda _: obj


def _nargs(func):
    return len(signature(func).parameters)


def _master(comm):
    return get_MPI_params_from_comm(comm)[2]


def _bcast(obj, comm):
    return obj if comm is None else comm.bcast(obj, root=0)


def _history_from(d):
    h = EnergyHistory()
    for t, v in zip(d["time_stamps"], d["energy_values"]):
        h.append((t, v))
    return h


def _normal_initialize(mf, domain, std=0.1):
    """optimize_kl.py:735-747: keys of `domain` missing from the mean start at
    N(0, std^2)"""
    if MultiDomain.union([domain, mf.domain]) != domain:
        raise RuntimeError(f"Domain of MultiField and final domain are not compatible\n"
                           f"MultiField domain:\n{mf.domain}\nFinal domain:\n{domain}")
    diff = set(domain.keys()) - set(mf.domain.keys())
    if not diff:
        return mf if mf.domain is domain else MultiField.from_dict({k: mf[k] for k in domain.keys()}, domain)
    fld = from_random(makeDomain({k: domain[k] for k in diff}), std=std)
    res = mf.unite(fld)
    myassert(res.domain == domain)
    return res


def _single_value_sample_list(fld, comm):
    if _master(comm):
        return SampleList([fld], comm=comm, domain=fld.domain)
    return SampleList([], comm=comm, domain=fld.domain)


def _clear_stem(base):
    import glob
    import os
    for f in glob.glob(glob.escape(base) + ".*.npz"):
        tail = f[len(base) + 1:-4]
        if tail == "mean" or tail.isdigit():
            os.remove(f)


def _export_operators(out, stem, ops, sl):
    """mean / std (several samples) or the single sample of each exported
    operator on the samples, as <out>/<name>/<stem>.npz (the reference writes
    HDF5 / FITS when h5py / astropy are installed, optimize_kl.py:465-498)"""
    for name, op in ops.items():
        if isinstance(op.domain, MultiDomain) and not all(k in sl.domain.keys() for k in op.domain.keys()):
            continue
        if sl.n_samples > 1:
            m, v = sl.sample_stat(lambda s: op(s.extract(op.domain) if isinstance(s, MultiField) else s))
            arrs = {"mean": np.asarray(m.val.cpu().numpy()), "std": np.sqrt(np.asarray(v.val.cpu().numpy()))}
        else:
            s = sl.local_item(0) if sl.n_local_samples else None
            if s is None:
                continue
            r = op(s.extract(op.domain) if isinstance(s, MultiField) else s)
            arrs = {"sample": np.asarray(r.val.cpu().numpy())}
        if _master(sl.comm):
            np.savez(join(out, name, stem + ".npz"), **arrs)
