"""MIOpen find database for the BASELINE configs on MI355X (gfx950, 256 CUs).

The critic and generator convolutions run on MIOpen in immediate mode
(``torch.backends.cudnn.benchmark = False``): without a find-db entry MIOpen
picks a solver by heuristic.  ``scaled-mmd-gan_amd/miopen_db/`` holds the
find results of ``tools/gpu_find.sh`` (``cudnn.benchmark`` on the bench
workload: every applicable solver timed per conv problem, e.g. the 1x1
512 -> 1024 shortcut at 8x8 runs 0.07 ms on an implicit-GEMM XDLOPS solver vs
0.36 ms on the heuristic's Winograd).  With the db, immediate mode takes the
measured-fastest solver: +1.4 % images/s on the SNResNet-64 step, with no
search at run time.

MIOpen writes to its user db, so ``install()`` copies the committed files to
a per-process directory and points ``MIOPEN_USER_DB_PATH`` at it -- unless the
user set that variable (or ``SMMD_MIOPEN_DB=0``).  It must run before the
first convolution (MIOpen reads the variable at its first db access).  The
file names carry the MIOpen version and the device (gfx950, 0x100 CUs);
another version or device simply finds no matching file and keeps its
heuristic.
"""
from __future__ import annotations

import glob
import os
import shutil
import tempfile

DB_DIR = os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))),
                      'miopen_db')


def install():
    """Point MIOpen at a writable copy of the committed find db; returns the
    directory used, or None when left to the user / disabled."""
    if os.environ.get('MIOPEN_USER_DB_PATH') or os.environ.get('SMMD_MIOPEN_DB', '1') == '0':
        return None
    files = glob.glob(os.path.join(DB_DIR, '*.txt'))
    if not files:
        return None
    dst = tempfile.mkdtemp(prefix='smmd_miopen_db_')
    for f in files:
        shutil.copy(f, dst)
    os.environ['MIOPEN_USER_DB_PATH'] = dst
    return dst
