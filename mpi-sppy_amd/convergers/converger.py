"""Converger contract (mirrors ``mpisppy/convergers/converger.py:17-40``)."""
import abc


class Converger(abc.ABC):
    def __init__(self, opt):
        self.conv = None
        self._opt = opt

    @abc.abstractmethod
    def is_converged(self):
        pass

    def post_everything(self):
        pass
