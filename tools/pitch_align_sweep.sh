# Padded-row alignment for short / large rows (tools/pitch_probe.py cases 2, 3:
# C4 u16 .T with 20000-B rows, f32 rows of 4400 B), padded vs dense per setting.
set -o pipefail
for a in 128 256 512 1024; do
  echo "== align $a"
  BOLT_AMD_PITCH_ALIGN=$a BOLT_AMD_PITCH_PAD_DIV=4 timeout -k 10 300 python tools/pitch_probe.py 5 1,2,3 || exit 1
done
