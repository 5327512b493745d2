"""PH extension initialising W and/or xbar from csv (``mpisppy/utils/wxbarreader.py``).

PHoptions keys: ``init_W_fname`` (file, or directory with
``init_separate_W_files``), ``init_Xbar_fname``.  Missing files raise
(the reference quits); W / prox are re-enabled for Iter0 as the reference does.
"""
import os

from . import wxbarutils


class WXBarReader:
    def __init__(self, ph, rank=None, n_proc=None):
        rank = ph.cylinder_rank if rank is None else rank
        o = ph.PHoptions
        sep_files = o.get("init_separate_W_files", False)
        w_fname = o.get("init_W_fname")
        x_fname = o.get("init_Xbar_fname")
        if w_fname is not None and not os.path.exists(w_fname):
            raise FileNotFoundError(("Cannot find path " if sep_files else "Cannot find file ") + w_fname)
        if x_fname is not None and not os.path.exists(x_fname):
            raise FileNotFoundError("Cannot find file " + x_fname)
        if x_fname is None and w_fname is None and rank == 0:
            print("Warning: no input files provided to WXBarReader. "
                  "W and Xbar will be initialized to their default values.")
        self.PHB = ph
        self.cylinder_rank = rank
        self.w_fname, self.x_fname, self.sep_files = w_fname, x_fname, sep_files

    def pre_iter0(self, *args):
        """wxbarreader.py:76-85."""
        if self.w_fname:
            wxbarutils.set_W_from_file(self.w_fname, self.PHB, self.cylinder_rank,
                                       sep_files=self.sep_files)
            self.PHB._reenable_W()
        if self.x_fname:
            wxbarutils.set_xbar_from_file(self.x_fname, self.PHB)
            self.PHB._reenable_prox()

    def post_iter0(self, *args):
        pass

    def miditer(self, *args):
        pass

    def enditer(self, *args):
        pass

    def post_everything(self, *args):
        pass
