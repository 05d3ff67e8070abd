"""Extension hook contract (mirrors ``mpisppy/extensions/extension.py:12-169``).

The engine calls these at the same points of Iter0 / iterk_loop / solve_loop as
the reference.  Per-subproblem ``pre_solve`` / ``post_solve`` are called (for
every local scenario, around the batched solve) only when a subclass overrides
them, so the common no-hook case costs nothing per scenario.
"""


class Extension:
    def __init__(self, spopt_object):
        self.opt = spopt_object

    def pre_solve(self, subproblem):
        pass

    def post_solve(self, subproblem, results):
        return results

    def pre_solve_loop(self):
        pass

    def post_solve_loop(self):
        pass

    def pre_iter0(self):
        pass

    def post_iter0(self):
        pass

    def post_iter0_after_sync(self):
        pass

    def miditer(self):
        pass

    def enditer(self):
        pass

    def enditer_after_sync(self):
        pass

    def post_everything(self):
        pass


class MultiExtension(Extension):
    """Call several extensions in order (extension.py:113-169)."""

    def __init__(self, ph, ext_classes):
        super().__init__(ph)
        self.extdict = {cls.__name__: cls(ph) for cls in ext_classes}

    def _all(self, name, *a):
        for e in self.extdict.values():
            getattr(e, name)(*a)

    def pre_solve(self, subproblem):
        self._all("pre_solve", subproblem)

    def post_solve(self, subproblem, results):
        for e in self.extdict.values():
            results = e.post_solve(subproblem, results)
        return results

    def pre_solve_loop(self):
        self._all("pre_solve_loop")

    def post_solve_loop(self):
        self._all("post_solve_loop")

    def pre_iter0(self):
        self._all("pre_iter0")

    def post_iter0(self):
        self._all("post_iter0")

    def post_iter0_after_sync(self):
        self._all("post_iter0_after_sync")

    def miditer(self):
        self._all("miditer")

    def enditer(self):
        self._all("enditer")

    def enditer_after_sync(self):
        self._all("enditer_after_sync")

    def post_everything(self):
        self._all("post_everything")
