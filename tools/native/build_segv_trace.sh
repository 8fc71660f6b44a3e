#!/bin/bash
# builds tools/native/libsegv_trace.so (diagnosis helper, see segv_trace.c)
cd "$(dirname "$0")" && gcc -O1 -g -shared -fPIC -rdynamic -o libsegv_trace.so segv_trace.c
