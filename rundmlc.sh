#!/bin/bash
/usr/local/bin/python -m dmlc_core_amd.parallel.launch.container echo hi
