"""Scenario creators of the reference examples, rebuilt on LinearModel."""
