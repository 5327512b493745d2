"""PH driver (mirrors ``mpisppy/opt/ph.py``)."""
from .. import phbase


class PH(phbase.PHBase):
    """PH.  See PHBase for the list of args."""

    def ph_main(self, finalize=True):
        """``opt/ph.py:26-72``: PH_Prep -> subproblem_creation -> Iter0 ->
        iterk_loop -> post_loops.  Returns (conv, Eobj, trivial_bound);
        Eobj is None when finalize is False."""
        verbose = self.PHoptions["verbose"]
        self.PH_Prep()
        self.subproblem_creation(verbose)
        trivial_bound = self.Iter0()
        if self.PHoptions.get("asynchronousPH", False):
            raise RuntimeError("asynchronousPH is deprecated; use APH")
        self.iterk_loop()
        if finalize:
            Eobj = self.post_loops(self.PH_extensions)
        else:
            Eobj = None
        return self.conv, Eobj, trivial_bound
