"""ORACLE — TEST INFRASTRUCTURE ONLY (see oracle/ipm_oracle.c).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product package mcp_amd/ never does.
"""
