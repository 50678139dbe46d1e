"""GPU worker: one process per GPU (or TP group) -- claims jobs from the core's
lease queue and executes them in-process on its own engines."""
