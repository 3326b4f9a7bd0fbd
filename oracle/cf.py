"""Oracle: SimpleCorrelatedField (src/library/correlated_fields_simple.py:38-170)
value, Jacobian-vector product and vector-Jacobian product, in numpy.
TEST INFRASTRUCTURE ONLY.

Latent vectors are dicts {key: ndarray}.  The amplitude follows the
reference's operator order literally:
  fluct  = LognormalTransform(fluctuations)                 normal_operators.py:55-75
  slope  = vslope * NormalTransform(loglogavgslope)         correlated_fields_simple.py:88-91
  asp    = xi_spec * sig_flex * sqrt(shift + sig_asp)       :93-117
  a      = Normalization(slope + SlopeRemover(TwoLog(asp)))  :118-119, correlated_fields.py:91-201
  a      = maskzm * fluct * a (+ zeromode) ; a *= total_volume   :120-127
  s      = offset_mean + HT(a[pindex] * xi)                 :129-134
"""
import numpy as np

from . import dispatch, geometry


def lognormal_moments(mean, sigma):
    """utilities.lognormal_moments (src/utilities.py:405-418)"""
    logsigma = np.sqrt(np.log1p((sigma / mean) ** 2))
    logmean = np.log(mean) - logsigma ** 2 / 2
    return float(logmean), float(logsigma)


class CFOracle:
    def __init__(self, shape, offset_mean, offset_std, fluctuations, flexibility, asperity,
                 loglogavgslope, prefix="", convention="non_canonical_hartley"):
        self.shape = tuple(shape)
        self.hdist = geometry.harmonic_distances(shape)
        self.pindex, self.kl, _ = geometry.power_space(self.shape, self.hdist)
        self.B = len(self.kl)
        self.p = prefix
        self.offset_mean = offset_mean
        self.conv = convention
        self.fl_m = lognormal_moments(*fluctuations)
        self.sl = (float(loglogavgslope[0]), float(loglogavgslope[1]))
        self.flex_m = None if flexibility is None else lognormal_moments(*flexibility)
        self.asp_m = None if asperity is None else lognormal_moments(*asperity)
        self.zm_m = None if offset_std is None else lognormal_moments(*offset_std)
        logk = np.log(self.kl[1:])
        rel = logk - logk[0]
        self.vslope = np.insert(rel, 0, 0.)
        self.sc = self.vslope / self.vslope[-1]
        self.lv = logk[1:] - logk[:-1]
        self.mult = np.bincount(self.pindex.ravel(), minlength=self.B).astype(np.float64)
        self.mult[0] = 0.
        self.total_volume = 1.0  # default position distances 1/n
        self.c_h = float(np.prod(self.hdist))

    def k(self, name):
        return self.p + name

    # --------------------------------------------------------------- helpers
    def _twolog(self, x):
        """_TwoLogIntegrations.apply TIMES (correlated_fields.py:127-143)"""
        c = np.cumsum(x[1])
        cp = np.r_[0., c[:-1]]
        t = (c + cp) / 2 * self.lv + x[0]
        return np.r_[0., 0., np.cumsum(t)]

    def _twolog_adj(self, g):
        """(correlated_fields.py:144-155): numpy overlapping in-place add keeps old values"""
        x = g.copy()
        res = np.zeros((2, len(g) - 2))
        x[2:] = np.cumsum(x[2:][::-1])[::-1]
        res[0] += x[2:]
        x[2:] *= self.lv / 2.
        x[1:-1] += x[2:]
        res[1] += np.cumsum(x[2:][::-1])[::-1]
        return res

    def _sr(self, x):
        return x - x[-1] * self.sc

    def _sr_adj(self, x):
        r = x.copy()
        r[-1] -= np.sum(x * self.sc)
        return r

    # --------------------------------------------------------------- model
    def amplitude(self, lat):
        c = {}
        fl = np.exp(self.fl_m[0] + self.fl_m[1] * lat[self.k("fluctuations")])
        a = self.vslope * (self.sl[0] + self.sl[1] * lat[self.k("loglogavgslope")])
        if self.flex_m is not None:
            flex = np.exp(self.flex_m[0] + self.flex_m[1] * lat[self.k("flexibility")])
            vflex = np.sqrt(self.lv)
            sig_flex = np.vstack([vflex, vflex]) * flex
            shift = np.vstack([self.lv ** 2 / 12., np.ones_like(self.lv)])
            if self.asp_m is not None:
                asp = np.exp(self.asp_m[0] + self.asp_m[1] * lat[self.k("asperity")])
                sig_asp = np.vstack([np.full_like(self.lv, asp), np.zeros_like(self.lv)])
                sq = np.sqrt(shift + sig_asp)
                c["asp"] = asp
            else:
                sq = np.sqrt(shift)
            xs = lat[self.k("spectrum")]
            a = a + self._sr(self._twolog(xs * sig_flex * sq))
            c.update(flex=flex, sig_flex=sig_flex, sq=sq, xs=xs)
        spec = np.exp(a)
        S = np.sum(self.mult * spec)
        An = np.sqrt(spec * (1. / S))
        amp = fl * An
        amp[0] = 0.
        if self.zm_m is not None:
            zm = np.exp(self.zm_m[0] + self.zm_m[1] * lat[self.k("zeromode")])
            amp[0] += zm
            c["zm"] = zm
        amp = amp * self.total_volume
        c.update(fl=fl, spec=spec, S=S, An=An)
        return amp, c

    def value(self, lat):
        amp, _ = self.amplitude(lat)
        s = self.c_h * dispatch.hartley(amp[self.pindex] * lat[self.k("xi")], convention=self.conv)
        if self.offset_mean is not None:
            s = s + self.offset_mean
        return s

    def amp_jvp(self, lat, c, t):
        dfl = c["fl"] * self.fl_m[1] * t[self.k("fluctuations")]
        da = self.vslope * self.sl[1] * t[self.k("loglogavgslope")]
        if self.flex_m is not None:
            dflex = c["flex"] * self.flex_m[1] * t[self.k("flexibility")]
            dsig = np.vstack([np.sqrt(self.lv), np.sqrt(self.lv)]) * dflex
            dat = t[self.k("spectrum")] * c["sig_flex"] * c["sq"] + c["xs"] * dsig * c["sq"]
            if self.asp_m is not None:
                dasp = c["asp"] * self.asp_m[1] * t[self.k("asperity")]
                dsq = np.vstack([dasp / (2 * c["sq"][0]), np.zeros_like(self.lv)])
                dat = dat + c["xs"] * c["sig_flex"] * dsq
            da = da + self._sr(self._twolog(dat))
        dS = np.sum(self.mult * c["spec"] * da)
        dAn = c["An"] * (da / 2. - dS / (2. * c["S"]))
        dam = dfl * c["An"] + c["fl"] * dAn
        dam[0] = 0.
        if self.zm_m is not None:
            dam[0] += c["zm"] * self.zm_m[1] * t[self.k("zeromode")]
        return dam * self.total_volume

    def amp_vjp(self, lat, c, g):
        out = {}
        g = g * self.total_volume
        if self.zm_m is not None:
            out[self.k("zeromode")] = np.asarray(c["zm"] * self.zm_m[1] * g[0])
        gm = g.copy()
        gm[0] = 0.
        out[self.k("fluctuations")] = np.asarray(c["fl"] * self.fl_m[1] * np.sum(gm * c["An"]))
        gAn = c["fl"] * gm
        ga = c["An"] * gAn / 2. - self.mult * c["spec"] * np.sum(gAn * c["An"]) / (2. * c["S"])
        out[self.k("loglogavgslope")] = np.asarray(self.sl[1] * np.sum(self.vslope * ga))
        if self.flex_m is not None:
            gat = self._twolog_adj(self._sr_adj(ga))
            out[self.k("spectrum")] = gat * c["sig_flex"] * c["sq"]
            gsig = gat * c["xs"] * c["sq"]
            out[self.k("flexibility")] = np.asarray(
                c["flex"] * self.flex_m[1] * np.sum(gsig * np.sqrt(self.lv)[None, :]))
            if self.asp_m is not None:
                gsq0 = gat[0] * c["xs"][0] * c["sig_flex"][0]
                out[self.k("asperity")] = np.asarray(
                    c["asp"] * self.asp_m[1] * np.sum(gsq0 / (2 * c["sq"][0])))
        return out

    def jvp(self, lat, t):
        amp, c = self.amplitude(lat)
        da = self.amp_jvp(lat, c, t)
        u = amp[self.pindex] * t[self.k("xi")] + lat[self.k("xi")] * da[self.pindex]
        return self.c_h * dispatch.hartley(u, convention=self.conv)

    def vjp(self, lat, g):
        amp, c = self.amplitude(lat)
        v = self.c_h * dispatch.hartley(g, convention=self.conv)
        ga = geometry.power_collect(lat[self.k("xi")] * v, self.pindex, self.B)
        out = self.amp_vjp(lat, c, ga)
        out[self.k("xi")] = amp[self.pindex] * v
        return out
