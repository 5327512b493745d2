"""PH extensions of the build (the reference's mpisppy/extensions)."""
