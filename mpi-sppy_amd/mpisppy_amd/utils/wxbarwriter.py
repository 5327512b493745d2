"""PH extension writing W and/or xbar to csv after PH (``mpisppy/utils/wxbarwriter.py``).

PHoptions keys: ``W_fname`` (file, or directory with ``separate_W_files``),
``Xbar_fname``.  Files are appended to, as in the reference.
"""
import os

from . import wxbarutils


class WXBarWriter:
    def __init__(self, ph, rank=None, n_proc=None):
        rank = ph.cylinder_rank if rank is None else rank
        o = ph.PHoptions
        w_fname = o.get("W_fname")
        x_fname = o.get("Xbar_fname")
        sep_files = o.get("separate_W_files", False)
        if x_fname is None and w_fname is None and rank == 0:
            print("Warning: no output files provided to WXBarWriter. No values will be saved.")
        if w_fname and not sep_files and os.path.exists(w_fname) and rank == 0:
            print(f"Warning: specified W_fname ({w_fname}) already exists. "
                  "Results will be appended to this file.")
        elif w_fname and sep_files and not os.path.exists(w_fname) and rank == 0:
            print(f"Warning: path {w_fname} does not exist. Creating...")
            os.makedirs(w_fname, exist_ok=True)
        if x_fname and os.path.exists(x_fname) and rank == 0:
            print(f"Warning: specified Xbar_fname ({x_fname}) already exists. "
                  "Results will be appended to this file.")
        self.PHB = ph
        self.cylinder_rank = rank
        self.w_fname, self.x_fname, self.sep_files = w_fname, x_fname, sep_files

    def pre_iter0(self, *args):
        pass

    def post_iter0(self, *args):
        pass

    def miditer(self, *args):
        pass

    def enditer(self, *args):
        pass

    def post_everything(self, *args):
        """wxbarwriter.py:96-103."""
        if self.w_fname:
            wxbarutils.write_W_to_file(self.PHB, self.w_fname, sep_files=self.sep_files)
        if self.x_fname:
            wxbarutils.write_xbar_to_file(self.PHB, self.x_fname)
