"""TEST INFRASTRUCTURE ONLY: the CPU oracle (see oracle/oracle.c). Never imported by the product."""
