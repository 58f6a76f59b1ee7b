"""monitor/metrics"""
