"""Cylinder-side users of the batched solver (hub/spoke transport: see DESIGN.md)."""
SPOKE_SLEEP_TIME = 0.1
