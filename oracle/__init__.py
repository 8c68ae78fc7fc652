"""CPU oracle — test infrastructure only (see oracle/model.py header). Parity unpinned: the
reference (Keras/TF) cannot run here and ships no golden vectors."""
