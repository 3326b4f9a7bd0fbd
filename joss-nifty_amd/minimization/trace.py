"""Decision trace of the sampling path (a test hook, off by default).

When ``TRACE`` is a list, the controllers, the NewtonCG driver and the line
search append what they decide, so that a test can hold the build's decisions
(CG iteration counts, Newton steps, line-search trial steps) to the
reference's, per sample, on the per-sample and on the batched geoVI path:

  (("lin", pair), (it, value))     a check of a linear sampling CG controller
  (("newton", sample), (it, value)) a check of a NewtonCG outer controller
  (("dir", sample), (it, value))   a check of a Newton-direction CG controller
  (("trial", sample), None)        a line search starts
  (("trial", sample), alpha)       the line search asks for the energy at alpha
  (("trialE", sample), None / value) the same stream: line search starts,
                                   the energy value found at each trial step
  (("trialD", sample), (value, dd)) a directional derivative the line search
                                   asked for, with the energy value there

``it`` is the controller's iteration number (0 at its start, so every solve
begins with it == 0), ``sample`` the index of the refined sample among the
rank's local samples, ``pair`` the index of the linear solve among the rank's
drawn right-hand sides.  Reading ``energy.value`` for the trace costs a
reduction and a host sync per check; nothing is recorded (or computed) while
``TRACE`` is None.
"""
TRACE = None


def active():
    return TRACE is not None


def emit(tag, value):
    if TRACE is not None and tag is not None:
        TRACE.append((tag, value))


def tag(obj, t):
    """attach trace tag ``t`` to a controller (no-op while tracing is off)"""
    if TRACE is not None:
        obj._trace_tag = t
    return obj


def solves(values):
    """split a controller's (it, value) stream into solves: [[value, ...], ...]"""
    out = []
    for it, v in values:
        if it == 0:
            out.append([])
        out[-1].append(v)
    return out


def trials(values):
    """split a trial stream into line searches: [[alpha, ...], ...]"""
    out = []
    for a in values:
        if a is None:
            out.append([])
        else:
            out[-1].append(a)
    return out


def by_tag(events=None):
    """{tag: [values in order]}"""
    out = {}
    for t, v in (TRACE if events is None else events):
        out.setdefault(t, []).append(v)
    return out
