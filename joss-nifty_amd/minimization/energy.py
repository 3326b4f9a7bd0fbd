"""Energy base class (src/minimization/energy.py:24-136)."""


class Energy:
    def __init__(self, position):
        self._position = position
        self._gradnorm = None

    def at(self, position):
        return self.__class__(position)

    @property
    def position(self):
        return self._position

    @property
    def value(self):
        raise NotImplementedError

    @property
    def gradient(self):
        raise NotImplementedError

    @property
    def gradient_norm(self):
        if self._gradnorm is None:
            self._gradnorm = self.gradient.norm()
        return self._gradnorm

    @property
    def metric(self):
        raise NotImplementedError

    def apply_metric(self, x):
        raise NotImplementedError

    def longest_step(self, direction):
        return None
