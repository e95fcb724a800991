#!/bin/bash
# Host code under sanitizers (race detection; CPU only, this container):
#   ASan + UBSan build (make SAN=address,undefined): every scene loader (.ecs, .xml, .obj/.mtl,
#   Collada .dae — the hand-written XML DOM), the PNG / baseline-JPEG / PPM decoders, the image
#   writers, the oracle, and a seeded mutation fuzz of each parser's inputs;
#   TSan build (make SAN=thread): the shard hub's host phases from several threads (mutex,
#   condition variable, deadlines).
# usage: tools/run_sanitizers.sh [log] [fuzz mutations per file]
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LOG=${1:-$ROOT/profiles/r05/sanitizers_r05.txt}
NFUZZ=${2:-300}
mkdir -p "$(dirname "$LOG")"
cd "$ROOT/yulio-raytracer_amd" || exit 1
make -j8 -s SAN=address,undefined BUILD=build_san LIB=lib_san all san > /tmp/san_build.log 2>&1 || { tail -20 /tmp/san_build.log; exit 1; }
make -j8 -s SAN=thread BUILD=build_tsan LIB=lib_tsan all san > /tmp/tsan_build.log 2>&1 || { tail -20 /tmp/tsan_build.log; exit 1; }
cd "$ROOT" || exit 1
# generated inputs: the Collada test scene (tests/dae_scene.py), the Frederick St. stand-in
# .dae, the Sponza stand-in .xml and the other generated scenes the tests use
GEN=$(mktemp -d /tmp/san_inputs.XXXX)
python3 - "$GEN" <<'PY'
import sys
from pathlib import Path
root = Path.cwd()
sys.path[:0] = [str(root), str(root / "yulio-raytracer_amd"), str(root / "tests")]
import dae_scene
from yrt import frederick, standin
out = Path(sys.argv[1])
dae_scene.write(out)
frederick.write_dae()
standin.write_xml()
PY
SCENES=$(ls scenes/*.ecs scenes/*.xml scenes/samples/*.ecs scenes/samples/*.xml scenes/_generated/*.xml \
  scenes/_generated/*.ecs scenes/_generated/*.dae "$GEN"/*.dae)
IMAGES=$(ls scenes/*.png scenes/*.ppm scenes/Sponza/*.JPG scenes/frederick/*.jpg scenes/frederick/*.jpeg scenes/frederick/*.png)
FUZZ="$GEN/room.dae scenes/cornell_box.obj scenes/cornell_box.mtl scenes/cornell_box.ecs scenes/cornell_box_spheres.xml \
  scenes/test_stereo.xml scenes/test_stereo_view.ecs scenes/materials_lights.ecs scenes/samples/sphere_motion.xml \
  scenes/logo.png scenes/frederick/material_77.png scenes/frederick/Kitchen_Sink.jpg \
  scenes/frederick/Metal_Aluminum_Anodized.jpg scenes/frederick/Brick_Antique_01.jpg scenes/lines.ppm"
export ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=0:detect_stack_use_after_return=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
export TSAN_OPTIONS=halt_on_error=1:second_deadlock_stack=1
export TMPDIR=${TMPDIR:-/tmp}
rc=0
t0=$SECONDS
step() { echo "   ($((SECONDS - t0)) s so far)"; }
{
  echo "# tools/run_sanitizers.sh on $(date -u +%Y-%m-%dT%H:%MZ), $(git rev-parse --short HEAD)"
  echo "# clang $(/opt/rocm/llvm/bin/clang++ --version | head -1); fuzz: $NFUZZ seeded mutations per file"
  echo "## ASan + UBSan: scene loaders, BVH build, frame export, oracle thumbnails"
  timeout 1800 yulio-raytracer_amd/lib_san/san_driver scenes $SCENES 2>&1 || rc=1
  step
  echo "## ASan + UBSan: image decoders and writers"
  timeout 900 yulio-raytracer_amd/lib_san/san_driver images $IMAGES 2>&1 || rc=1
  step
  echo "## ASan + UBSan: seeded mutation fuzz (seed 5)"
  timeout 3000 yulio-raytracer_amd/lib_san/san_driver fuzz 5 "$NFUZZ" $FUZZ 2>&1 || rc=1
  step
  echo "## ASan + UBSan: shard hub"
  timeout 600 yulio-raytracer_amd/lib_san/san_driver hub 6 2>&1 || rc=1
  step
  echo "## TSan: shard hub (threads)"
  timeout 900 yulio-raytracer_amd/lib_tsan/san_driver hub 12 2>&1 || rc=1
  step
  echo "## TSan: scene loaders (the BVH builder's threads)"
  timeout 1800 yulio-raytracer_amd/lib_tsan/san_driver scenes scenes/cornell_box_spheres.ecs scenes/_generated/sponza_standin.xml "$GEN"/room.dae 2>&1 || rc=1
  step
  echo "## exit status $rc (0: no sanitizer report, every step returned)"
} > "$LOG" 2>&1
rm -rf "$GEN"
tail -3 "$LOG"
exit $rc
