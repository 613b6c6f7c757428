#!/bin/bash
# every list-bind shape once (tools/list_bind_probe.py), for tools/gpu_ab_lib.sh
for s in shuffled_each reversed shuffled_same sorted; do
  SHAPE=$s python -u tools/list_bind_probe.py || exit 1
done
