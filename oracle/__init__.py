"""Test-infrastructure oracle package (see oracle/oracle.py). Never imported by hydra_amd."""
