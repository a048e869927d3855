#!/bin/sh
# Builds the N-API addon (node-gyp is not available offline): mtreplay.node links
# ../libmtreplay.so and ../libmtsnapdec.so (built by fluidframework_amd/build.py) through an $ORIGIN rpath.
set -e
HERE=$(cd "$(dirname "$0")" && pwd)
NODE_INC=${NODE_INC:-/usr/include/node}
g++ -std=c++17 -O2 -Wall -shared -fPIC -DNODE_GYP_MODULE_NAME=mtreplay -I"$NODE_INC" \
    "$HERE/binding.cc" -o "$HERE/mtreplay.node.tmp" -L"$HERE/.." -lmtreplay -lmtsnapdec -Wl,-rpath,'$ORIGIN/..'
mv "$HERE/mtreplay.node.tmp" "$HERE/mtreplay.node"
