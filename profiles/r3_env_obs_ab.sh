set -o pipefail
for L in "" variants/libmuz_obs1.so variants/libmuz_obs2.so; do
  echo "== lib ${L:-in-tree}"
  if [ -n "$L" ]; then export MUZ_LIB=$PWD/exploring-muzero-on-dog_amd/$L; else unset MUZ_LIB; fi
  timeout -k 10 200 python profiles/env_breakdown.py 2>&1 | grep "B=" || exit 1
done
