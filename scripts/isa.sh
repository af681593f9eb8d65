#!/bin/bash
# Device ISA of one kernel (gfx950): scripts/isa.sh SRC.hip MANGLED_SUBSTR > out.s
set -e
SRC=$1; K=$2
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -munsafe-fp-atomics -x hip \
  --cuda-device-only -S "$SRC" -o /tmp/isa_all.s
python3 - "$K" <<'PY'
import sys
s = open('/tmp/isa_all.s').read()
k = sys.argv[1]
i = s.index(k + ':') if k + ':' in s else s.index(k)
e = s.index('.Lfunc_end', i)
print(s[i:e])
PY
