"""TEST INFRASTRUCTURE ONLY -- see oracle/oracle.py."""
