#!/bin/bash
# Builds a timing variant of the product library from a SNAPSHOT of the
# sources (so edits made while hipcc runs cannot mix two layouts of the Dev
# record into one library): scripts/build_variant.sh NAME "DEFS"
# -> go-libp2p-pubsub_amd/build/libgossip_engine_var_NAME.so
set -e
cd "$(dirname "$0")/.."
NAME=$1
DEFS=$2
TMP=$(mktemp -d /tmp/gsvar.XXXXXX)
mkdir -p "$TMP/go-libp2p-pubsub_amd"
cp -r include "$TMP/"
cp -r go-libp2p-pubsub_amd/csrc go-libp2p-pubsub_amd/Makefile "$TMP/go-libp2p-pubsub_amd/"
make -s -C "$TMP/go-libp2p-pubsub_amd" var NAME="$NAME" DEFS="$DEFS"
mkdir -p go-libp2p-pubsub_amd/build
cp "$TMP/go-libp2p-pubsub_amd/build/libgossip_engine_var_$NAME.so" go-libp2p-pubsub_amd/build/
rm -rf "$TMP"
echo "built go-libp2p-pubsub_amd/build/libgossip_engine_var_$NAME.so"
