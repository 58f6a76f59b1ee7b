"""monitor/analysis"""
