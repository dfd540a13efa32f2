"""Drop-in package name of the reference (``nf``), served by normalizingflow_amd."""
