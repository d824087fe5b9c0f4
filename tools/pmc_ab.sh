#!/bin/bash
# Same PMC sets over two tune variants: bash tools/pmc_ab.sh <tag> "<varA>" "<varB>" "<set1>" ["<set2>"...]
set -e
tag=$1; va=$2; vb=$3; shift 3
bash tools/pmc_pass.sh ${tag}_a "$va" "$@"
bash tools/pmc_pass.sh ${tag}_b "$vb" "$@"
