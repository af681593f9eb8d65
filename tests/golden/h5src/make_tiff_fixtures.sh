#!/bin/bash
# Regenerates tests/golden/*.tif with libtiff (gcc against the image's
# /opt/conda libtiff; not needed at test time).
set -e
D=$(cd "$(dirname "$0")" && pwd)
B=$(mktemp -d)
gcc -O1 -I/opt/conda/include -o $B/mk "$D/make_tiff_fixtures.c" -L/opt/conda/lib -ltiff
LD_LIBRARY_PATH=/opt/conda/lib $B/mk "$D/.."
rm -rf $B
