#!/bin/bash
# Builds the product library of a committed revision (timing A/B against the
# working tree): scripts/build_ref.sh NAME REF [DEFS]
# -> go-libp2p-pubsub_amd/build/libgossip_engine_var_NAME.so
set -e
cd "$(dirname "$0")/.."
NAME=$1
REF=$2
DEFS=$3
TMP=$(mktemp -d /tmp/gsref.XXXXXX)
git archive "$REF" include go-libp2p-pubsub_amd/csrc go-libp2p-pubsub_amd/Makefile | tar -x -C "$TMP"
make -s -C "$TMP/go-libp2p-pubsub_amd" var NAME="$NAME" DEFS="$DEFS"
mkdir -p go-libp2p-pubsub_amd/build
cp "$TMP/go-libp2p-pubsub_amd/build/libgossip_engine_var_$NAME.so" go-libp2p-pubsub_amd/build/
rm -rf "$TMP"
echo "built go-libp2p-pubsub_amd/build/libgossip_engine_var_$NAME.so ($REF)"
