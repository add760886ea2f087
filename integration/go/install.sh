#!/bin/bash
# Installs the MI355X Go seam into a gnark checkout (the reference tree layout):
#
#   integration/go/install.sh <gnark-checkout>
#
#   gm/                    -> backend/accel/mi355x/gm          (cgo binding; build tag icicle)
#   icicle_bn254/          -> backend/groth16/bn254/icicle      (replaces icicle.go, noicicle.go,
#                                                                provingkey.go, doc.go; keeps marshal_test.go)
#   icicle_bls12377/       -> backend/groth16/bls12-377/icicle  (new GPU hook for the second curve)
#   plonk_bls12377/*.go    -> backend/plonk/bls12-377           (kzg.Commit / FFT hook)
#
# and applies the three patches with patch -p1 (no fuzz):
#   icicle_bls12377/groth16.go.diff  backend/groth16/groth16.go   (BLS12-377 dispatch, like :200-204)
#   plonk_bls12377/prove.go.diff     backend/plonk/bls12-377/prove.go
#   solver_levelhook.diff            constraint/solver/options.go, constraint/{bn254,bls12-377}/solver.go
#
# The #cgo lines of gm.go are rewritten to this repository's include/ and
# gnark-icicle_amd/ (libgnark_mi355x.so).  Then:
#   go test ./...                                   # default build: no cgo, CPU provers
#   go test -tags icicle ./backend/...              # GPU provers (WithIcicleAcceleration)
#   go build -tags icicle,mi355x_levelhook ./...    # + a/b/c staged to the GPU during Solve
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REPO="$(cd "$HERE/../.." && pwd)"
G="${1:?usage: install.sh <gnark-checkout>}"
[ -f "$G/backend/groth16/groth16.go" ] || { echo "not a gnark checkout: $G" >&2; exit 1; }

# dry-run every patch first: nothing is touched unless all apply
for p in icicle_bls12377/groth16.go.diff plonk_bls12377/prove.go.diff solver_levelhook.diff; do
  patch -d "$G" -p1 -F0 --dry-run -s -i "$HERE/$p" >/dev/null || { echo "patch does not apply: $p" >&2; exit 1; }
done

mkdir -p "$G/backend/accel/mi355x/gm"
cp "$HERE"/gm/*.go "$G/backend/accel/mi355x/gm/"
sed -i -e "s#^\#cgo CFLAGS: .*#\#cgo CFLAGS: -I$REPO/include#" \
       -e "s#^\#cgo LDFLAGS: .*#\#cgo LDFLAGS: -L$REPO/gnark-icicle_amd -lgnark_mi355x -Wl,-rpath,$REPO/gnark-icicle_amd#" \
       "$G/backend/accel/mi355x/gm/gm.go"

D="$G/backend/groth16/bn254/icicle"
rm -f "$D/icicle.go" "$D/noicicle.go" "$D/provingkey.go" "$D/doc.go"
cp "$HERE"/icicle_bn254/*.go "$D/"

mkdir -p "$G/backend/groth16/bls12-377/icicle"
cp "$HERE"/icicle_bls12377/*.go "$G/backend/groth16/bls12-377/icicle/"

cp "$HERE"/plonk_bls12377/*.go "$G/backend/plonk/bls12-377/"

for p in icicle_bls12377/groth16.go.diff plonk_bls12377/prove.go.diff solver_levelhook.diff; do
  patch -d "$G" -p1 -F0 -s -i "$HERE/$p"
done
echo "installed into $G"
