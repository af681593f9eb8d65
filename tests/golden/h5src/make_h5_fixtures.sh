#!/bin/bash
# Regenerates tests/golden/*.h5 with the real HDF5 C library (gcc against the
# image's /opt/conda HDF5 1.10.6; not needed at test time).
set -e
D=$(cd "$(dirname "$0")" && pwd)
B=$(mktemp -d)
gcc -O1 -I/opt/conda/include -o $B/mk "$D/make_h5_fixtures.c" -L/opt/conda/lib -lhdf5 -lm
LD_LIBRARY_PATH=/opt/conda/lib $B/mk "$D/.."
rm -rf $B
