"""oracle -- CPU restatement of WJGiles/Dorknet's hot path.  TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this
package, and only as the checker / the reported CPU baseline -- never as the thing that
is measured or shipped.  The product package (dorknet_amd) never imports it and has no
CPU fallback.

  ref.py       numpy restatement of every hot-path function (fp32 or fp64), with
               reference file:line citations
  net.py       layer / residual / network / SGD-momentum objects built on ref.py
  cpu_path.py  the reference's *CPU* path: C/OpenMP restatements of its Cython kernels
               (csrc/dorknet_oracle.c, built by the Makefile) + numpy BLAS (np.dot)
  models.py    ResNet-18-depsep and MNISTNet (examples/) as oracle networks

PARITY UNPINNED: the reference has no tests, golden vectors or fixtures, and importing /
running the reference was denied.  The restatement is pinned instead by
an independent oracle (torch CPU conv2d / batch_norm / autograd), analytic known-answer
tests, and committed seeded fixtures (tests/golden).
"""
