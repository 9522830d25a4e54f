#!/bin/bash
# builds tools/_bin/mt_records (tools/mt_records.c) against the in-tree engine; run here, it travels with the snapshot
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/_bin
gcc -O2 -Wall -pthread -Iinclude tools/mt_records.c -Lpicotls_amd/_lib -lptls_mi355x \
    -Wl,-rpath,'$ORIGIN/../../picotls_amd/_lib' -o tools/_bin/mt_records
