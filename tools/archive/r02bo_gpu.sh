#!/bin/bash
# r02bo: -R 6 / -R 8 solve groups vs shipped (libs built on the CPU side into lib_ab/R6, lib_ab/R8)
AB_TAG=r02bo AB_LIBS="cur R6 R8" bash tools/ab_libs.sh
