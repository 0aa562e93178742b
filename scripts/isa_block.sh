#!/bin/bash
# print one basic block of a kernel in a hipcc -S listing: isa_block.sh file.s kernel-prefix label
awk -v K="$2" -v L="$3:" 'index($0,K)==1&&/:/{f=1} f&&$1==L{p=1} p{print} p&&/s_cbranch/{exit}' "$1" | grep -v "^\s*;"
